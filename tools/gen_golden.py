"""Generate golden fixtures from the REFERENCE ITSELF (build container only).

Imports the reference modules by file path from /root/reference (read-only,
never copied), runs them on CPU with seeded inputs and the synthetic weight
recipe of ``itsd.weights``, and writes small ``.npz`` fixtures (inputs and
expected outputs only) to ``tests/golden/``. The reference's sampler prints
every step; stdout is silenced while it runs.

    python tools/gen_golden.py            # regenerate everything
    python tools/gen_golden.py archC_eps  # only the named fixture(s) of the "extra" group

The GPU box never runs this (it has no /root/reference).
"""
from __future__ import annotations

import contextlib
import hashlib
import importlib.util
import io
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)

import itsd  # noqa: E402
import dataclasses  # noqa: E402

from itsd.arch import ARCH_A, ARCH_C, ARCH_TINY, ARCH_TINY_CFG  # noqa: E402
from itsd.weights import synthetic_state_dict  # noqa: E402


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m


def _stub_torchvision():
    tv = types.ModuleType("torchvision")
    tr = types.ModuleType("torchvision.transforms")
    tr.Resize = lambda *a, **k: None
    tv.transforms = tr
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tr)


def sha(t: torch.Tensor) -> str:
    return hashlib.sha256(t.contiguous().numpy().tobytes()).hexdigest()[:16]


def save(name, **arrs):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)) for k, v in arrs.items()})
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def ref_ddpm(M, a, sd):
    net = M.UNet(T=a.T, ch=a.ch, ch_mult=list(a.ch_mult), attn=list(a.attn), num_res_blocks=a.num_res_blocks,
                 dropout=0.0)
    net.load_state_dict(sd)
    return net.eval()


def ref_cfg(MC, a, sd):
    net = MC.UNet(T=a.T, num_labels=a.num_labels, ch=a.ch, ch_mult=list(a.ch_mult),
                  num_res_blocks=a.num_res_blocks, dropout=0.0)
    net.load_state_dict(sd)
    return net.eval()


def noise_sequence(seed, shape, T):
    """The draws the reference sampler consumes: randn(x_T) then randn_like for
    steps T-1..1 (Diffusion.py:96), all from the default CPU generator."""
    torch.manual_seed(seed)
    xT = torch.randn(shape)
    zs = [torch.randn(shape) for _ in range(T - 1)]
    return xT, torch.stack(zs) if zs else torch.zeros((0,) + tuple(shape))


def extra(M, MC, only):
    """Full-size fixtures of the configs beyond C2 (outputs only; weights = recipe seed 0)."""
    with torch.no_grad():
        if not only or "archC_eps" in only:
            # C3: the CFG UNet (MainCondition.py:10-13) at 32 px; attention at S = 1024 .. 1
            a = ARCH_C
            sd = synthetic_state_dict(a, seed=0)
            net = ref_cfg(MC, a, sd)
            g = torch.Generator().manual_seed(21)
            x = torch.randn(2, 3, 32, 32, generator=g)
            t = torch.tensor([10, 900])
            lab = torch.tensor([4, 0])
            save("archC_eps", x=x, t=t, labels=lab, eps=net(x, t, lab))
            del net, sd
        if not only or "archA64_eps" in only:
            # C4: Arch A with img_size 64 (attention at S = 256)
            a = dataclasses.replace(ARCH_A, img_size=64)
            sd = synthetic_state_dict(a, seed=0)
            net = ref_ddpm(M, a, sd)
            g = torch.Generator().manual_seed(22)
            x = torch.randn(2, 3, 64, 64, generator=g)
            t = torch.tensor([3, 700])
            save("archA64_eps", x=x, t=t, eps=net(x, t))
        if not only or "archA256_eps" in only:
            # the reference's ImageNet resolution (example/imagenet_ep50_bs1024_T1000_lr1e-4.sh:30,
            # config/inference_config.yaml img_size 256): attention at S = 4096, d = 384
            a = dataclasses.replace(ARCH_A, img_size=256)
            sd = synthetic_state_dict(a, seed=0)
            net = ref_ddpm(M, a, sd)
            g = torch.Generator().manual_seed(23)
            x = torch.randn(1, 3, 256, 256, generator=g)
            t = torch.tensor([400])
            save("archA256_eps", x=x, t=t, eps=net(x, t))


def main():
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[1:]
    torch.set_num_threads(8)
    M = _load("ref_model", "Diffusion/Model.py")
    D = _load("ref_diffusion", "Diffusion/Diffusion.py")
    MC = _load("ref_model_cond", "DiffusionFreeGuidence/ModelCondition.py")
    DC = _load("ref_diffusion_cond", "DiffusionFreeGuidence/DiffusionCondition.py")
    S = _load("ref_search", "search/search_algorithm.py")
    if only:
        torch.set_num_threads(8)
        extra(M, MC, only)
        print("torch", torch.__version__)
        return
    _stub_torchvision()
    with contextlib.redirect_stdout(io.StringIO()):
        V = _load("ref_verifier", "search/verifier.py")

    # 1. schedules (Diffusion.py:57-65, :76)
    sched = {}
    for (T, b1, bT) in [(1000, 1e-4, 0.02), (1000, 1e-4, 0.028), (3000, 1e-4, 0.02), (10, 1e-4, 0.02)]:
        smp = D.GaussianDiffusionSampler(torch.nn.Identity(), b1, bT, T)
        var = torch.cat([smp.posterior_var[1:2], smp.betas[1:]])
        tag = f"T{T}_b{bT}"
        sched[tag + "_betas"] = smp.betas
        sched[tag + "_coeff1"] = smp.coeff1
        sched[tag + "_coeff2"] = smp.coeff2
        sched[tag + "_posterior_var"] = smp.posterior_var
        sched[tag + "_var"] = var
    save("schedules", **sched)

    with torch.no_grad():
        # 2. tiny DDPM eps (Model.py:265-285)
        a = ARCH_TINY
        sd = synthetic_state_dict(a, seed=0)
        net = ref_ddpm(M, a, sd)
        g = torch.Generator().manual_seed(1)
        x = torch.randn(4, 3, 32, 32, generator=g)
        t = torch.tensor([0, 1, 499, 999])
        save("tiny_ddpm_eps", x=x, t=t, eps=net(x, t), temb=net.time_embedding(t))

        # 3. tiny DDPM sampler trajectory, T=10 (Diffusion.py:84-102)
        T = 10
        smp = D.GaussianDiffusionSampler(net, 1e-4, 0.02, T)
        xT, zs = noise_sequence(7, (2, 3, 32, 32), T)
        torch.manual_seed(7)
        xT2 = torch.randn(2, 3, 32, 32)
        with contextlib.redirect_stdout(io.StringIO()):
            x0 = smp(xT2)
        assert torch.equal(xT, xT2)
        save("tiny_ddpm_traj", seed=7, T=T, x_T=xT, noise=zs, x0=x0, noise_sha=sha(zs))

        # 4. tiny CFG eps and a guided T=6 trajectory (ModelCondition.py:206-235, DiffusionCondition.py:79-105)
        a = ARCH_TINY_CFG
        sdc = synthetic_state_dict(a, seed=0)
        netc = ref_cfg(MC, a, sdc)
        x = torch.randn(4, 3, 32, 32, generator=g)
        t = torch.tensor([0, 3, 500, 999])
        lab = torch.tensor([1, 5, 10, 0])
        save("tiny_cfg_eps", x=x, t=t, labels=lab, eps=netc(x, t, lab))
        T = 6
        smpc = DC.GaussianDiffusionSampler(netc, 1e-4, 0.028, T, w=1.8)
        xT, zs = noise_sequence(11, (2, 3, 32, 32), T)
        torch.manual_seed(11)
        xT2 = torch.randn(2, 3, 32, 32)
        lab2 = torch.tensor([3, 7])
        with contextlib.redirect_stdout(io.StringIO()):
            x0 = smpc(xT2, lab2)
        save("tiny_cfg_traj", seed=11, T=T, w=1.8, labels=lab2, x_T=xT, noise=zs, x0=x0)

        # 5. full Arch A eps at 3 timesteps and a T=20 trajectory (outputs only; weights = recipe seed 0)
        a = ARCH_A
        sdA = synthetic_state_dict(a, seed=0)
        netA = ref_ddpm(M, a, sdA)
        x = torch.randn(3, 3, 32, 32, generator=g)
        t = torch.tensor([0, 500, 999])
        save("archA_eps", x=x, t=t, eps=netA(x, t))
        T = 20
        smpA = D.GaussianDiffusionSampler(netA, 1e-4, 0.02, T)
        xT, zs = noise_sequence(5, (2, 3, 32, 32), T)
        torch.manual_seed(5)
        with contextlib.redirect_stdout(io.StringIO()):
            x0 = smpA(torch.randn(2, 3, 32, 32))
        save("archA_traj", seed=5, T=T, x0=x0, noise_sha=sha(zs))

        # 6. verifiers (verifier.py:45-66, 223-248, 262-287)
        gv = torch.Generator().manual_seed(3)
        cases = {
            "b1_neg": torch.randn(1, 3, 32, 32, generator=gv).clamp(-1, 1),
            "b4_neg": torch.randn(4, 3, 32, 32, generator=gv).clamp(-1, 1),
            "b4_pos": torch.rand(4, 3, 32, 32, generator=gv),
            "b2_neg": (torch.randn(2, 3, 32, 32, generator=gv) * 0.3).clamp(-1, 1),
        }
        ov, sv, av = V.OracleVerifier(), V.SelfSupervisedVerifier(), V.AestheticPredictor(device="cpu")
        vres = {}
        for k, im in cases.items():
            vres[k + "_images"] = im
            vres[k + "_oracle"] = np.float64(ov.score(im))
            vres[k + "_selfsup"] = np.float64(sv.score(im))
            vres[k + "_aesthetic"] = np.float64(av.score(im))
        save("verifiers", **vres)

        # 7. search outcomes on the tiny UNet, T=5 (search_algorithm.py)
        T = 5
        smp5 = D.GaussianDiffusionSampler(net, 1e-4, 0.02, T)

        def denoise_fn(noise, show_progress=False, **kw):
            with contextlib.redirect_stdout(io.StringIO()):
                return smp5(noise)

        rec = []

        def verifier_fn(images, **kw):
            s = ov.score(images)
            rec.append(s)
            return s

        shape = (1, 3, 32, 32)
        torch.manual_seed(0)
        rs = S.RandomSearch(n_candidates=4)
        bn, bs = rs.search(shape, denoise_fn, verifier_fn, device="cpu", verbose=False)
        res = {"random_best_noise": bn, "random_best_score": np.float64(bs), "random_scores": np.array(rec),
               "random_nfes": rs.nfes}
        rec.clear()
        torch.manual_seed(1)
        init = torch.randn(shape)
        zo = S.ZeroOrderSearch(n_neighbors=3, lambda_radius=0.95, n_iterations=2)
        bn, bs, h = zo.search(init, denoise_fn, verifier_fn, device="cpu", verbose=False)
        res.update(zo_init=init, zo_best_noise=bn, zo_best_score=np.float64(bs), zo_scores=np.array(h["scores"]),
                   zo_nfes=zo.nfes, zo_seed_after_init=1)
        rec.clear()
        torch.manual_seed(2)
        init = torch.randn(shape)
        ps = S.PathSearch(n_paths=3, injection_step=400, noise_scale=0.1)
        bn, bs, h = ps.search(init, denoise_fn, verifier_fn, timesteps=T, device="cpu", verbose=False)
        res.update(path_init=init, path_best_noise=bn, path_best_score=np.float64(bs),
                   path_scores=np.array(h["scores"]), path_nfes=ps.nfes)
        save("search_T5", **res)
    extra(M, MC, None)
    print("torch", torch.__version__)


if __name__ == "__main__":
    main()
