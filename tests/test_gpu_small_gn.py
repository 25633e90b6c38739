"""conv_small with its consumer GroupNorm(+SiLU) in the epilogue (option small_gn; ModelCondition.py ResBlock /
AttnBlock GroupNorms at the CFG model's 2x2 and 1x1 levels): where a GroupNorm reads the output
of the conv right before it and nothing else, conv_small's whole-image tiles already hold every (image, group) of
that output, so the epilogue finalizes the group statistics exactly as gn_apply_kernel does (the same per-channel slot
sums, the same fp64 order and 8-lane butterfly, the same coefficient expressions) and writes silu(GN(out)) beside
out; the GroupNorm launch is skipped.

  * bit-identical to the unfused path (small_gn 0) for the C3 guided batch (2N = 64), a ragged batch whose 1x1-level
    tile is part-empty (10) and one spanning two 1x1-level tiles (100); deterministic; within bf16 tolerance of the
    oracle;
  * the census loses one GroupNorm launch per fused pair (23 of 37 at 2N = 64: the up path's GroupNorms over
    torch.cat(h, skip) keep theirs).
"""
import pytest
import torch

from oracle import ref_cpu as R
from itsd import runtime as rt
from itsd.arch import ARCH_C
from itsd.model import CondUNet
from itsd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
REL_L2_BF16 = 2e-2

_NET = {}


def _net():
    if "c" not in _NET:
        c = ARCH_C
        net = CondUNet(c.T, c.num_labels, c.ch, c.ch_mult, c.num_res_blocks, 0.0, img_size=32, precision="bf16")
        net.load_state_dict(synthetic_state_dict(c, 0))
        _NET["c"] = net.to("cuda:0")
    return _NET["c"]


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


def _eps(net, x, t, lab, v):
    rt.set_option("small_gn", v)
    try:
        return net(x, t, lab).float().cpu()
    finally:
        rt.set_option("small_gn", 1)


@pytest.mark.parametrize("n", [64, 10, 100])
def test_small_gn_bit_identical_to_gn_launch(n):
    net = _net()
    gen = torch.Generator().manual_seed(7300 + n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, ARCH_C.T, (n,), generator=gen)
    lab = torch.arange(n) % (ARCH_C.num_labels + 1)
    xd, td, ld = x.cuda(), t.cuda(), lab.cuda()
    fused = _eps(net, xd, td, ld, 1)
    again = _eps(net, xd, td, ld, 1)
    plain = _eps(net, xd, td, ld, 0)
    assert torch.isfinite(fused).all()
    assert torch.equal(fused, again)
    assert torch.equal(fused, plain), _rel_l2(fused, plain)
    idx = [0, n - 1]
    c = ARCH_C
    with torch.no_grad():
        ref = R.unet_forward(synthetic_state_dict(c, 0), x[idx], t[idx], c.ch, c.ch_mult, c.attn, c.num_res_blocks,
                             labels=lab[idx], cfg=True)
    d = _rel_l2(fused[idx], ref)
    print(f"n={n}: fused GroupNorm output == GroupNorm launch bit for bit; vs oracle rel-L2 {d:.2e}")
    assert d < REL_L2_BF16


def test_small_gn_removes_groupnorm_launches():
    net = _net()
    n = 64
    x = torch.randn(n, 3, 32, 32, device="cuda")
    t = torch.full((n,), 500, dtype=torch.int32, device="cuda")
    nat = net.native(n)
    counts = {}
    for v in (0, 1):
        rt.set_option("small_gn", v)
        try:
            ops = nat.profile_ops(x, t)
        finally:
            rt.set_option("small_gn", 1)
        counts[v] = (sum(o["kind"] == "gn" for o in ops), len(ops))
    print(f"2N = {n}: GroupNorm launches {counts[0][0]} -> {counts[1][0]}, launches {counts[0][1]} -> {counts[1][1]}")
    assert counts[1][0] < counts[0][0] and counts[0][1] - counts[1][1] == counts[0][0] - counts[1][0]
    assert counts[0][0] - counts[1][0] >= 20
