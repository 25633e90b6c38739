"""attn_block_kernel: the whole AttnBlock (Model.py:145-164: GroupNorm, q|k|v 1x1, softmax(q k^T /
sqrt(C)) v, proj 1x1, residual) of Arch A's 8x8 level in one launch, against the unfused path
(gn_apply + q|k|v conv + attn_mfma_kernel + proj conv, attn_fuse=0 at create) and the oracle.
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


def _net(fuse):
    a = ARCH_A
    rt.set_option("attn_fuse", fuse)
    try:
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16")
        net.load_state_dict(synthetic_state_dict(a, 0))
        net.to("cuda:0")
        net.native(8)  # the handle is built (and the option read) here
    finally:
        rt.set_option("attn_fuse", 1)
    return net


@pytest.mark.parametrize("n", [8, 256])
def test_fused_attnblock_vs_unfused_and_oracle(n):
    fused, plain = _net(1), _net(0)
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
    net = _net(1)
    n = 16
    x = torch.randn(n, 3, 32, 32, device="cuda")
    t = torch.full((n,), 500, dtype=torch.int32, device="cuda")
    ops = net.native(n).profile_ops(x, t)
    at8 = [o for o in ops if o["H"] == 8]
    kinds = [o["kind"] for o in at8]
    assert kinds.count("attnblock") == 5 and "attn" not in kinds and "gn" not in kinds, kinds
    assert all("attn_block_kernel" in o["kernel"] for o in at8 if o["kind"] == "attnblock")
