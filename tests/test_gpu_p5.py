"""conv3x3_gn_p5_kernel: the split-K persistent fused GroupNorm+SiLU+conv3x3 of the 8x8 / 4x4
levels (Model.py:170-174,179-184), against the oracle and against the other fused kernels.

  * every forced K-slice count (1, 2, 3, 8) is deterministic run to run -- the last-arriving slice
    sums the partials in slice order, whatever the arrival order -- and within 1.5e-2 relative L2
    of the unsplit run and 2e-2 of the oracle (bf16);
  * at 8x8 the p5 tiles (128 px, two images) forced on agree with p4's (256 px, four images);
  * ragged batches (images past the batch in the last tile) and the census (the 4x4 level runs the
    fused kernel: no materialised GroupNorm before its convs but the attention one).
"""
import pytest
import torch

from oracle import ref_cpu as R
from itsd import runtime as rt
from itsd.arch import ARCH_A
from itsd.model import UNet
from itsd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
REL_L2_BF16 = 2e-2
_DEFAULTS = {"p5": 1, "p5_split": 0}


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


def _net():
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16")
    net.load_state_dict(synthetic_state_dict(a, 0))
    return net.to("cuda:0")


def _eps(net, x, t, **opts):
    try:
        for k, v in opts.items():
            rt.set_option(k, v)
        return net(x, t).float().cpu()
    finally:
        for k, v in _DEFAULTS.items():
            rt.set_option(k, v)


def _oracle(x, t):
    a = ARCH_A
    with torch.no_grad():
        return R.unet_forward(synthetic_state_dict(a, 0), x, t, a.ch, a.ch_mult, a.attn, a.num_res_blocks)


@pytest.mark.parametrize("n", [64, 5])
def test_p5_split_counts_deterministic_and_vs_oracle(n):
    net = _net()
    gen = torch.Generator().manual_seed(500 + n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    xd, td = x.cuda(), t.cuda()
    base = _eps(net, xd, td, p5=2, p5_split=1)
    idx = [0, n // 2, n - 1]
    ref = _oracle(x[idx], t[idx])
    assert _rel_l2(base[idx], ref) < REL_L2_BF16
    for S in (2, 3, 8):
        a = _eps(net, xd, td, p5=2, p5_split=S)
        b = _eps(net, xd, td, p5=2, p5_split=S)
        assert torch.equal(a, b), S
        d = _rel_l2(a, base)
        print(f"n={n} split {S}: rel-L2 vs unsplit {d:.2e}, vs oracle {_rel_l2(a[idx], ref):.2e}")
        assert d < 1.5e-2 and _rel_l2(a[idx], ref) < REL_L2_BF16


def test_p5_vs_p4_full_batch():
    """N = 256: every fused level on p4 (p5=0: 256-pixel tiles, several per block) vs p5 forced
    on at every level (p5=2: 128-pixel tiles of whole images at 8x8, of 8 / 4 image rows in the
    halo "rows" mode at 16x16 / 32x32)."""
    net = _net()
    gen = torch.Generator().manual_seed(77)
    x = torch.randn(256, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (256,), generator=gen)
    xd, td = x.cuda(), t.cuda()
    p4 = _eps(net, xd, td, p5=0)
    p5 = _eps(net, xd, td, p5=2)
    assert torch.isfinite(p5).all()
    d = _rel_l2(p5, p4)
    ref = _oracle(x[[0, 255]], t[[0, 255]])
    print(f"p5 vs p4 (N=256): rel-L2 {d:.2e}; vs oracle {_rel_l2(p5[[0, 255]], ref):.2e}")
    assert d < 1.5e-2 and _rel_l2(p5[[0, 255]], ref) < REL_L2_BF16


def test_p5_small_batch_vs_128px_kernels():
    """N = 32 (the 8-GPU shard of N = 256): p5 takes every level (auto) -- against p5=0 (the
    128-pixel conv3x3_gn_kernel at 32x32 / 16x16, p4 / the 128-px kernel at 8x8; 4x4 stays p5)."""
    net = _net()
    gen = torch.Generator().manual_seed(32)
    x = torch.randn(32, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (32,), generator=gen)
    xd, td = x.cuda(), t.cuda()
    ops = net.native(32).profile_ops(xd, td.to(torch.int32))
    p5_levels = sorted({o["H"] for o in ops if "conv3x3_gn_p5_kernel" in o["kernel"]})
    assert p5_levels == [4, 8, 16, 32], p5_levels
    auto = _eps(net, xd, td)
    old = _eps(net, xd, td, p5=0)
    ref = _oracle(x[[0, 31]], t[[0, 31]])
    print(f"N=32 p5 vs 128-px kernels: rel-L2 {_rel_l2(auto, old):.2e}; vs oracle {_rel_l2(auto[[0, 31]], ref):.2e}")
    assert _rel_l2(auto, old) < 1.5e-2 and _rel_l2(auto[[0, 31]], ref) < REL_L2_BF16


def test_p5_census_4x4_level_fused():
    net = _net()
    n = 16
    x = torch.randn(n, 3, 32, 32, device="cuda")
    t = torch.full((n,), 500, dtype=torch.int32, device="cuda")
    ops = net.native(n).profile_ops(x, t)
    at4 = [o for o in ops if o["H"] == 4]
    p5 = [o for o in at4 if "conv3x3_gn_p5_kernel" in o["kernel"]]
    gn = [o for o in at4 if o["kind"] == "gn"]
    print({o["kernel"] for o in at4})
    assert len(p5) == 14  # block1 + block2 of the 7 ResBlocks at 4x4 (2 down, 2 middle, 3 up)
    assert len(gn) == 1   # the middle AttnBlock's GroupNorm (materialised for the q|k|v conv)


def test_p5_gn_fold_vs_gn_coef_launches():
    """gn_fold: conv3x3_gn_p5_kernel reduces its input's statistics slabs to group mean / rstd itself
    (fp64, as gn_coef_kernel) and the gn_coef launch before it is skipped; the forward equals the
    unfolded one to the last bits of the fp64 group sums (rel-L2 <= 1e-3)."""
    net = _net()
    n = 32
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    xd, td = x.cuda(), t.cuda()
    folded = _eps(net, xd, td)
    rt.set_option("gn_fold", 0)
    try:
        plain = _eps(net, xd, td)
        ops0 = net.native(n).profile_ops(xd, td.to(torch.int32))
    finally:
        rt.set_option("gn_fold", 1)
    ops1 = net.native(n).profile_ops(xd, td.to(torch.int32))
    c0 = sum(o["kind"] == "gncoef" for o in ops0)
    c1 = sum(o["kind"] == "gncoef" for o in ops1)
    print(f"gn_coef launches: {c0} unfolded, {c1} folded; rel-L2 {_rel_l2(folded, plain):.2e}")
    assert c1 < c0 - 30 and _rel_l2(folded, plain) < 1e-3
