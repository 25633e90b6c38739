"""conv3x3_gn_p5_kernel's split-K combine shared by every slice (option p5_dist, Model.py:170-174,179-184,
202-209): where each item has a block of its own, every slice of a tile waits for the tile's other slices and
finishes its own share of the tile's (pixel block, cout group) units -- the same slice order and the same
statistics tree as the last-arriving-slice combine, so the two forms are bit-identical:

  * the metric's shards and the batches around them (n = 8 / 16 / 32 / 64 / 256) and a ragged batch, auto plans
    (the cost model's slice counts and shortcut folds) and forced 3x3 slice counts 2 / 3 / 4 / 8 / 16, shared
    vs last arriver (p5_dist 2: the same plans) bit for bit, deterministic run to run, within bf16 tolerance of the
    oracle; and against the round-5 plans (p5_dist 0, the last arriver's cost model) within bf16 tolerance;
  * fail loudly: a hand-off wait that exhausts its poll bound (spin_bound 0) sets bit 1 of the status word and
    writes NaN, and the counters stay consistent for the next forward.
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
_DEFAULTS = {"p5_dist": 1, "p5_split": 0, "p5": 1, "p5_sc": 1, "p5_pub": 1, "p5_xl": 3}


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


_NET = {}


def _net():
    if "a" not in _NET:
        a = ARCH_A
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16")
        net.load_state_dict(synthetic_state_dict(a, 0))
        _NET["a"] = net.to("cuda:0")
    return _NET["a"]


def _eps(net, x, t, **opts):
    try:
        for k, v in opts.items():
            rt.set_option(k, v)
        return net(x, t).float().cpu()
    finally:
        for k, v in _DEFAULTS.items():
            rt.set_option(k, v)


def _inputs(n, seed):
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    return x, t


@pytest.mark.parametrize("n", [8, 16, 32, 64, 256, 5])
def test_shared_combine_bit_identical_auto(n):
    net = _net()
    x, t = _inputs(n, 6100 + n)
    xd, td = x.cuda(), t.cuda()
    shared = _eps(net, xd, td)
    again = _eps(net, xd, td)
    last = _eps(net, xd, td, p5_dist=2)
    assert torch.isfinite(shared).all()
    assert torch.equal(shared, again)
    assert torch.equal(shared, last), _rel_l2(shared, last)
    r5 = _eps(net, xd, td, p5_dist=0)
    assert _rel_l2(shared, r5) < 1.5e-2
    idx = [0, n - 1]
    ref = R.unet_forward(synthetic_state_dict(ARCH_A, 0), x[idx], t[idx], ARCH_A.ch, ARCH_A.ch_mult, ARCH_A.attn,
                         ARCH_A.num_res_blocks)
    d = _rel_l2(shared[idx], ref)
    print(f"n={n}: shared == last-arriver bit for bit; vs oracle rel-L2 {d:.2e}")
    assert d < REL_L2_BF16
    assert net.native(n).query("status") == 0


@pytest.mark.parametrize("n", [16, 32])
def test_shared_combine_bit_identical_forced_splits(n):
    """Forced 3x3 slice counts at every p5 level (p5=2: also the 32x32 / 16x16 levels, whose statistics slot is
    the whole 128-pixel tile: with more than 4 slices the slices past the 4 cout groups own no unit)."""
    net = _net()
    x, t = _inputs(n, 6200 + n)
    xd, td = x.cuda(), t.cuda()
    for S in (2, 3, 4, 8, 16):
        a = _eps(net, xd, td, p5=2, p5_split=S)
        b = _eps(net, xd, td, p5=2, p5_split=S, p5_dist=2)
        print(f"n={n} p5_split {S}: shared vs last arriver max|d| {(a - b).abs().max().item():.3e}")
        assert torch.isfinite(a).all() and torch.equal(a, b), S


def test_shared_combine_handoff_failure_is_loud():
    from itsd.diffusion import GaussianDiffusionSampler
    n = 32
    net = _net()
    x, t = _inputs(n, 6300)
    xd, td = x.cuda(), t.cuda()
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, 1000)
    rt.set_option("spin_bound", 0)
    try:
        eps = net(xd, td).float()
        status = net.native(n).query("status")
        assert status & 2, status
        assert torch.isnan(eps).any()
        with pytest.raises(rt.ItsdError) as ei:
            smp.run(xd.clone(), t_begin=999, t_end=998, seed=3)
        assert ei.value.code == rt.ITSD_ERR_HANDOFF and "conv3x3_gn_p5_kernel" in str(ei.value), ei.value
    finally:
        rt.set_option("spin_bound", 1 << 22)
    eps = net(xd, td).float().cpu()
    assert net.native(n).query("status") == 0 and torch.isfinite(eps).all()
    assert torch.equal(eps, _eps(net, xd, td, p5_dist=2))


@pytest.mark.parametrize("n", [8, 16, 32, 64, 256, 5])
def test_two_slice_publish_once_bit_identical(n):
    """(round 6, option p5_pub) The two-slice last-arriver combine with only the FIRST arriver storing its partial
    (arrival first; the last arriver adds the published partial to its own in registers: p0 + p1 == p1 + p0) against
    both slices storing theirs (round 5): bit for bit, auto plans and every p5 level forced onto two slices
    (p5 = 2, p5_split = 2, no shortcut fold, so every p5 launch takes the two-slice path); the counters stay
    consistent run to run."""
    net = _net()
    x, t = _inputs(n, 6400 + n)
    xd, td = x.cuda(), t.cuda()
    for opts in ({}, {"p5": 2, "p5_split": 2, "p5_sc": 0}):
        once = _eps(net, xd, td, **opts)
        again = _eps(net, xd, td, **opts)
        both = _eps(net, xd, td, p5_pub=0, **opts)
        assert torch.isfinite(once).all()
        assert torch.equal(once, again), opts
        assert torch.equal(once, both), (opts, _rel_l2(once, both))
        print(f"n={n} {opts}: publish-once == both-publish bit for bit")
    rt.set_option("p5_pub", 1)
    assert net.native(n).query("status") == 0


@pytest.mark.parametrize("n", [8, 16, 32, 64, 256, 5])
def test_xcd_local_exchange_bit_identical(n):
    """(round 6, option p5_xl) The split-K partials exchanged through one XCD's L2 (a tile's slices as adjacent
    items, plain stores and L1-bypassing loads, each slice's XCC_ID checked with its arrival) against the
    write-through exchange (p5_xl 0): bit for bit, for the shared combine at 8x8 / 16x16 (1), every eligible form (2:
    also the 4x4 level and the two-slice publish-once combine) and the shipped forms (3: 1 + the two-slice form at
    8x8 / 16x16 where K <= 3456), auto plans and forced two /
    four slices at every p5 level; the status word stays 0 (no tile's slices ran on two XCDs)."""
    net = _net()
    x, t = _inputs(n, 6500 + n)
    xd, td = x.cuda(), t.cuda()
    for opts in ({}, {"p5": 2, "p5_split": 2, "p5_sc": 0}, {"p5": 2, "p5_split": 4, "p5_sc": 0}):
        ref = _eps(net, xd, td, p5_xl=0, **opts)
        assert torch.isfinite(ref).all()
        for xl in (1, 2, 3):
            out = _eps(net, xd, td, p5_xl=xl, **opts)
            assert torch.equal(out, ref), (opts, xl, _rel_l2(out, ref))
            assert net.native(n).query("status") == 0, (opts, xl)
        print(f"n={n} {opts}: XCD-local exchange == write-through bit for bit")
