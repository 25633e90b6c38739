"""attn_block_kernel: the whole AttnBlock (Model.py:145-164: GroupNorm, q|k|v 1x1, softmax(q k^T /
sqrt(C)) v, proj 1x1, residual) of Arch A's 8x8 level (one image a block) in one launch, against the
unfused path (gn_apply + q|k|v conv + attn_mfma_kernel + proj conv, attn_fuse=0 at create) and the oracle;
attn_block_split_kernel (an image over G blocks) against it, and its fail-loud hand-off.
Both paths round hn, q / k / v, P and O to bf16; the sums run in other orders, so they agree
within 1.5e-2 relative L2 (bf16 tolerance) rather than bit for bit."""
import pytest
import torch

from oracle import ref_cpu as R
from itsd import runtime as rt
from itsd.arch import ARCH_A
from itsd.model import UNet
from itsd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


ATTN_FUSE_DEFAULT = 1  # shipped: fused at S = 64 (the 4x4 middle block runs the unfused ops)


def _net(fuse, n=8):
    """A UNet whose native handle (capacity >= n, so no later re-create with other options) is built
    under attn_fuse = fuse."""
    a = ARCH_A
    rt.set_option("attn_fuse", fuse)
    try:
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16")
        net.load_state_dict(synthetic_state_dict(a, 0))
        net.to("cuda:0")
        net.native(max(n, 8))  # the handle is built (and the option read) here
    finally:
        rt.set_option("attn_fuse", ATTN_FUSE_DEFAULT)
    return net


@pytest.mark.parametrize("n", [8, 256, 6, 13])
def test_fused_attnblock_vs_unfused_and_oracle(n):
    fused, plain = _net(1, n), _net(0, n)
    gen = torch.Generator().manual_seed(900 + n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    ef = fused(x.cuda(), t.cuda()).float().cpu()
    ep = plain(x.cuda(), t.cuda()).float().cpu()
    assert torch.equal(ef, fused(x.cuda(), t.cuda()).float().cpu())  # deterministic
    idx = [0, n - 1]
    a = ARCH_A
    with torch.no_grad():
        ref = R.unet_forward(synthetic_state_dict(a, 0), x[idx], t[idx], a.ch, a.ch_mult, a.attn, a.num_res_blocks)
    d = _rel_l2(ef, ep)
    print(f"n={n}: fused vs unfused AttnBlock rel-L2 {d:.2e}; vs oracle fused {_rel_l2(ef[idx], ref):.2e} "
          f"unfused {_rel_l2(ep[idx], ref):.2e}")
    assert d < 1.5e-2 and _rel_l2(ef[idx], ref) < 2e-2


def test_fused_attnblock_census():
    n = 16
    net = _net(1, n)
    x = torch.randn(n, 3, 32, 32, device="cuda")
    t = torch.full((n,), 500, dtype=torch.int32, device="cuda")
    ops = net.native(n).profile_ops(x, t)
    at8 = [o for o in ops if o["H"] == 8]
    kinds = [o["kind"] for o in at8]
    assert kinds.count("attnblock") == 5 and "attn" not in kinds and "gn" not in kinds, kinds
    assert all("attn_block_" in o["kernel"] for o in at8 if o["kind"] == "attnblock")
    # n = 16: the image's work spread over 6 blocks (16 x 6 <= 256 CUs)
    assert all("attn_block_split_kernel<384, 6>" in o["kernel"] for o in at8 if o["kind"] == "attnblock"), at8
    # the 4x4 middle block (S = 16, C = 512): the unfused ops (GroupNorm, q|k|v conv, attention, proj)
    at4 = [o["kind"] for o in ops if o["H"] == 4 and o["kind"] in ("attnblock", "attn", "gn")]
    assert at4 == ["gn", "attn"], at4


def _eps_with_split(net, x, t, split):
    rt.set_option("attn_split", split)
    try:
        return net(x.cuda(), t.cuda()).float().cpu()
    finally:
        rt.set_option("attn_split", 1)


@pytest.mark.parametrize("n", [8, 32, 64, 128])
def test_split_attnblock_vs_single_block_and_oracle(n):
    """attn_block_split_kernel (an image's AttnBlock over G = 6 / 4 / 2 blocks with two write-through
    hand-offs; auto G at n = 8 / 32: 6, 64: 4, 128: 2) against attn_block_kernel (one block per image,
    attn_split = 0) and the oracle. Only the score sum runs in another order (G partial sums): within
    bf16 tolerance of the single-block kernel, deterministic run to run; forced G = 2 / 4 / 6 at n = 8."""
    net = _net(ATTN_FUSE_DEFAULT, n)
    gen = torch.Generator().manual_seed(1300 + n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    single = _eps_with_split(net, x, t, 0)
    split = _eps_with_split(net, x, t, 1)
    assert torch.equal(split, _eps_with_split(net, x, t, 1))  # deterministic whichever block arrives last
    d = _rel_l2(split, single)
    idx = [0, n - 1]
    a = ARCH_A
    with torch.no_grad():
        ref = R.unet_forward(synthetic_state_dict(a, 0), x[idx], t[idx], a.ch, a.ch_mult, a.attn, a.num_res_blocks)
    e = _rel_l2(split[idx], ref)
    print(f"n={n}: split vs single-block AttnBlock rel-L2 {d:.2e}; split vs oracle {e:.2e}")
    assert d < 1e-2 and e < 2e-2
    if n == 8:
        for G in (2, 4, 6):
            dg = _rel_l2(_eps_with_split(net, x, t, G), single)
            print(f"  forced G={G}: rel-L2 vs single-block {dg:.2e}")
            assert dg < 1e-2



def test_split_attnblock_handoff_failure_is_loud():
    """Fail loudly (Diffusion.py:100's NaN assert is the reference's own contract): with the hand-off poll
    bound forced to 0 (option spin_bound, diagnostic), the blocks that reach attn_block_split_kernel's
    hand-offs first give up waiting for the other slices. They must not produce a silent wrong image: the
    forward's eps is NaN, itsd_unet_query "status" reads bit 0, and the sampler returns ITSD_ERR_HANDOFF
    naming the kernel. With the shipped bound the same calls succeed and the status word is clear."""
    from itsd.diffusion import GaussianDiffusionSampler
    n = 8
    net = _net(ATTN_FUSE_DEFAULT, n)
    gen = torch.Generator().manual_seed(77)
    x = torch.randn(n, 3, 32, 32, generator=gen).cuda()
    t = torch.randint(0, 1000, (n,), generator=gen).cuda()
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, 1000)
    rt.set_option("attn_split", 6)
    try:
        rt.set_option("spin_bound", 0)
        try:
            eps = net(x, t).float()
            status = net.native(n).query("status")
            assert status & 1, status
            assert torch.isnan(eps).any()
            with pytest.raises(rt.ItsdError) as ei:
                smp.run(x.clone(), t_begin=999, t_end=998, seed=3)
            assert ei.value.code == rt.ITSD_ERR_HANDOFF and "attn_block_split_kernel" in str(ei.value), ei.value
        finally:
            rt.set_option("spin_bound", 1 << 22)
        eps = net(x, t).float()
        assert net.native(n).query("status") == 0 and torch.isfinite(eps).all()
        y = x.clone()
        smp.run(y, t_begin=999, t_end=998, seed=3)
        assert torch.isfinite(y).all()
    finally:
        rt.set_option("attn_split", 1)
