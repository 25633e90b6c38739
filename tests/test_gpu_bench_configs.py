"""GPU parity at the sizes bench.py times ("pin every timed configuration").

The persistent kernels pick their tile schedule from the batch (tiles per block, split-K, the
attention grid), so every configuration the bench measures is compared with the oracle at the
bench's own batch, through the same sampler entry point the bench calls (``sampler.run`` in
Philox mode); the oracle (fp32, CPU) runs a few images spread over the batch, fed the same
counter-based noise (``R.philox_normal``, the restatement of the tail kernel's generator).

  bench line                      batch here                 check
  headline  Arch A, N = 256       256, 10-step window        x rel-L2 <= 3e-2 (3 images)
  sweep     N = 32 / 64 / 1024    forward                    eps rel-L2 <= 2e-2 (3-4 images)
  C3        Arch C CFG, N = 32    guided batch 2N = 64:      eps rel-L2 <= 2e-2; x rel-L2 <= 3e-2
                                  forward + 20-step window   (w = 1.8, betas (1e-4, 0.028))
  C4        64 px, N = 16         forward + 20-step window   eps 2e-2; x 3e-2
  C5        T = 3000, N = 128     20-step window t=2999..    x rel-L2 <= 3e-2
  (reference: MainCondition.py:10-21, example/imagenet_*.sh img_size, fine_tune_extended_T.py,
   Diffusion/Diffusion.py:84-102, DiffusionCondition.py:89-105)
"""
import dataclasses

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from itsd.arch import ARCH_A, ARCH_C
from itsd.diffusion import CondGaussianDiffusionSampler, GaussianDiffusionSampler
from itsd.model import CondUNet, UNet
from itsd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

REL_L2_EPS = 2e-2   # bf16 forward vs the fp32 oracle
REL_L2_TRAJ = 3e-2  # bf16 sampler window vs the fp32 oracle loop


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


def _net(a, seed=0):
    if a.cfg:
        net = CondUNet(a.T, a.num_labels, a.ch, a.ch_mult, a.num_res_blocks, 0.0, img_size=a.img_size,
                       precision="bf16")
    else:
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=a.img_size, precision="bf16")
    net.load_state_dict(synthetic_state_dict(a, seed))
    return net.to("cuda:0")


def _oracle3(a, sd):
    return lambda x, t, labels=None: R.unet_forward(sd, x, t, a.ch, a.ch_mult, a.attn, a.num_res_blocks,
                                                    labels=labels, cfg=a.cfg)


def _check_forward(a, n, idx, seed):
    """bf16 forward of a batch of n vs the oracle on images idx (random t per image)."""
    sd = synthetic_state_dict(a, 0)
    net = _net(a)
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, a.img_size, a.img_size, generator=gen)
    t = torch.randint(0, a.T, (n,), generator=gen)
    args = [x.cuda(), t.cuda()]
    lab = None
    if a.cfg:  # the guided batch: conditional half (labels 1..10), unconditional half (label 0)
        lab = torch.cat([torch.arange(n // 2) % 10 + 1, torch.zeros(n - n // 2, dtype=torch.long)])
        args.append(lab.cuda())
    eps = net(*args).float().cpu()
    ii = torch.tensor(idx)
    with torch.no_grad():
        ref = _oracle3(a, sd)(x[ii], t[ii], None if lab is None else lab[ii])
    errs = [_rel_l2(eps[i], ref[k]) for k, i in enumerate(idx)]
    print(f"{a.kind} {a.img_size}px n={n}: eps rel-L2 per image {['%.2e' % e for e in errs]}")
    for i, e in zip(idx, errs):
        assert e < REL_L2_EPS, (i, e)


def _check_window(a, n, idx, T, steps, beta_T=0.02, w=None, seed=5):
    """`steps` Philox-mode sampler steps from t = T-1 on a batch of n (the bench's call:
    sampler.run(x, t_begin, t_end, seed, clip=False)) vs the oracle loop on images idx."""
    sd = synthetic_state_dict(a, 0)
    net = _net(a)
    smp = (CondGaussianDiffusionSampler(net, 1e-4, beta_T, T, w=w) if a.cfg
           else GaussianDiffusionSampler(net, 1e-4, beta_T, T))
    gen = torch.Generator().manual_seed(1000 + n)
    x = torch.randn(n, 3, a.img_size, a.img_size, generator=gen)
    lab = (torch.arange(n) % 10 + 1) if a.cfg else None  # the bench's C3 labels
    t_begin, t_end = T - 1, T - steps
    got = smp.run(x.cuda().contiguous(), t_begin=t_begin, t_end=t_end, seed=seed, clip=False,
                  labels=None if lab is None else lab.cuda()).cpu()
    per = 3 * a.img_size * a.img_size
    s = R.schedule(1e-4, beta_T, T)
    ii = torch.tensor(idx)
    fw = _oracle3(a, sd)
    if a.cfg:
        model_fn = R.cfg_eps(fw, lab[ii], w)
    else:
        model_fn = lambda xx, tt: fw(xx, tt)

    def nf(step, xx):  # element o of candidate i: Philox index i * per + o (noise_offset 0)
        return torch.stack([R.philox_normal(seed, step, np.arange(i * per, (i + 1) * per)) for i in idx]
                           ).reshape(xx.shape)

    with torch.no_grad():
        ref = R.p_sample_loop(model_fn, x[ii], s, nf, t_begin=t_begin, t_end=t_end, clip=False)
    errs = [_rel_l2(got[i], ref[k]) for k, i in enumerate(idx)]
    print(f"{a.kind} {a.img_size}px n={n} T={T}: {steps}-step window rel-L2 {['%.2e' % e for e in errs]}")
    for i, e in zip(idx, errs):
        assert e < REL_L2_TRAJ, (i, e)


# ------------------------------------------------------------------------- headline and sweep
def test_headline_N256_window_vs_oracle():
    """The headline batch (N = 256, Arch A, T = 1000): 10 sampler steps of the bench's graph."""
    _check_window(ARCH_A, 256, [0, 129, 255], 1000, 10)


@pytest.mark.parametrize("n,idx", [(8, [0, 5, 7]), (16, [0, 9, 15]), (32, [0, 17, 31]), (64, [0, 40, 63]),
                                   (1024, [0, 333, 700, 1023])])
def test_sweep_batches_forward_vs_oracle(n, idx):
    """The N sweep (north_star N in {64, 256, 1024}; N = 32 is the 8-GPU shard of N = 256, N = 16 / 8 the 4- / 8-GPU
    shards of N = 64): the
    persistent convs' grids, the split-K small level and the attention grid at each batch."""
    _check_forward(ARCH_A, n, idx, seed=n)


# ------------------------------------------------------------------------- legs
def test_C3_cfg_guided_batch64_forward_vs_oracle():
    """C3's guided batch (Arch C, N_local = 32 -> 2N = 64, both label halves)."""
    _check_forward(ARCH_C, 64, [0, 21, 31, 32, 63], seed=3)


def test_C3_cfg_window_vs_oracle():
    """C3's sampler at its bench batch: CFG w = 1.8, betas (1e-4, 0.028), N = 32, 20 guided steps
    (40 UNet forwards of the 64-image guided batch) against the oracle's guided loop."""
    _check_window(ARCH_C, 32, [0, 31], 1000, 20, beta_T=0.028, w=1.8)


A64 = dataclasses.replace(ARCH_A, img_size=64)


def test_C4_64px_N16_forward_vs_oracle():
    _check_forward(A64, 16, [0, 9, 15], seed=4)


def test_C4_64px_N16_window_vs_oracle():
    """C4's 64x64 step (the ImageNet-64 UNet shape, example/imagenet_*.sh img_size) at its bench shard
    N = 16: 20 sampler steps t = 999..980 against the oracle loop (5 steps were too few)."""
    _check_window(A64, 16, [3, 15], 1000, 20)


def test_C5_T3000_N128_window_vs_oracle():
    """C5 (fine_tune_extended_T.py: T = 3000) at its bench shard N = 128: steps 2999..2980 in
    bf16 -- the parity of the path-search round's sampler (replaces a finiteness-only check)."""
    a = dataclasses.replace(ARCH_A, T=3000)
    _check_window(a, 128, [0, 64, 127], 3000, 20)
