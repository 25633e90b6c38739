"""The ResBlock's 1x1 shortcut folded into its block2 conv (Model.py:200-205: h = conv2(silu(GN(h))) +
shortcut(x)) as extra K slices of conv3x3_gn_p5_kernel (option p5_sc: 0 off, 1 auto, 2 wherever block2 runs
on p5): the shortcut slices stage x raw (no GroupNorm) and multiply its centre tap by the shortcut's weights;
the last-arriving slice sums every partial in slice order, so the fold is deterministic. The unfolded path
rounds the shortcut's output to bf16 before block2 adds it; the folded one accumulates it in fp32, so the two
agree within bf16 tolerance (rel-L2 1e-2), not bit for bit; both within 2e-2 of the oracle (fp32)."""
import pytest
import torch

from oracle import ref_cpu as R
from itsd import runtime as rt
from itsd.arch import ARCH_A
from itsd.model import UNet
from itsd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
REL_L2_BF16 = 2e-2
SC_DEFAULT = 1
N_SHORTCUTS = 15  # Arch A: the down blocks entering 16x16 / 8x8 / 4x4 and the 12 up blocks (concat inputs)


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


def _net():
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16")
    net.load_state_dict(synthetic_state_dict(a, 0))
    return net.to("cuda:0")


def _run(net, x, t, sc, census=False):
    rt.set_option("p5_sc", sc)
    try:
        eps = net(x, t).float().cpu()
        ops = net.native(x.shape[0]).profile_ops(x, t.to(torch.int32)) if census else None
        return eps, ops
    finally:
        rt.set_option("p5_sc", SC_DEFAULT)


@pytest.mark.parametrize("n", [32, 64, 5, 256])
def test_shortcut_fold_vs_unfolded_and_oracle(n):
    net = _net()
    gen = torch.Generator().manual_seed(2100 + n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    xd, td = x.cuda(), t.cuda()
    plain, ops0 = _run(net, xd, td, 0, census=True)
    always, ops2 = _run(net, xd, td, 2, census=True)
    again, _ = _run(net, xd, td, 2)
    auto, ops1 = _run(net, xd, td, 1, census=True)
    assert torch.equal(always, again)  # deterministic whichever slice arrives last
    idx = [0, n - 1]
    ref = R.unet_forward(synthetic_state_dict(ARCH_A, 0), x[idx], t[idx], ARCH_A.ch, ARCH_A.ch_mult, ARCH_A.attn,
                         ARCH_A.num_res_blocks)
    folded2, folded1 = len(ops0) - len(ops2), len(ops0) - len(ops1)
    d2, d1 = _rel_l2(always, plain), _rel_l2(auto, plain)
    print(f"n={n}: shortcuts folded always {folded2} / auto {folded1}; rel-L2 vs unfolded {d2:.2e} / {d1:.2e}; "
          f"vs oracle unfolded {_rel_l2(plain[idx], ref):.2e} always {_rel_l2(always[idx], ref):.2e}")
    # every launch the fold removes is a 1x1 conv (a shortcut); all 15 at n = 32 (every level on p5), the 4x4
    # level's 4 at n = 256 (its down block and 3 up blocks; the larger levels run p4)
    gone = {o["op"] for o in ops0} - {o["op"] for o in ops2}
    assert all(o["kind"] == "conv" and o["ks"] == 1 for o in ops0 if o["op"] in gone), gone
    assert len(gone) == folded2 and folded2 == {32: N_SHORTCUTS, 256: 4}.get(n, folded2) and folded2 > 0, folded2
    assert 0 <= folded1 <= folded2
    assert d2 < 1e-2 and d1 < 1e-2
    assert _rel_l2(always[idx], ref) < REL_L2_BF16 and _rel_l2(auto[idx], ref) < REL_L2_BF16


def test_shortcut_fold_with_forced_splits():
    """Forced 3x3 slice counts (p5_split) with the shortcut slices after them: deterministic and within bf16
    tolerance of the unfolded run."""
    net = _net()
    n = 16
    gen = torch.Generator().manual_seed(2200)
    x = torch.randn(n, 3, 32, 32, generator=gen).cuda()
    t = torch.randint(0, 1000, (n,), generator=gen).cuda()
    plain, _ = _run(net, x, t, 0)
    for S in (1, 3):
        rt.set_option("p5_split", S)
        try:
            a, _ = _run(net, x, t, 2)
            b, _ = _run(net, x, t, 2)
        finally:
            rt.set_option("p5_split", 0)
        d = _rel_l2(a, plain)
        print(f"p5_split {S}: folded vs unfolded rel-L2 {d:.2e}")
        assert torch.equal(a, b) and d < 1e-2
