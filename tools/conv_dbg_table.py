"""Per-conv timing with parts of the conv kernels switched off (itsd_set_option
"conv_dbg"; measurement only, the outputs are wrong while set): 1 no in-loop loads,
2 no MFMA, 4 no GN statistics, 8 no GN transform, 16 no epilogue.

    python tools/conv_dbg_table.py
"""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from itsd import runtime as rt
from itsd.arch import ARCH_A
from itsd.model import UNet
a = ARCH_A
net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss")
net.to("cuda:0")
nat = net.native(256)
x = torch.randn(256, 3, 32, 32, device="cuda")
t = torch.full((256,), 500, dtype=torch.int32, device="cuda")
DBG = (0, 3, 7, 15, 31, 16, 8, 4)
res = {}
for d in DBG:
    rt.set_option("conv_dbg", d)
    for _ in range(3):
        ops = nat.profile_ops(x, t)
    res[d] = ops
rt.set_option("conv_dbg", 0)
print(f"{'#':>3} {'kind':5} {'M':>7} {'N':>5} {'K':>5} {'H':>3} {'ks':>2} " + " ".join(f"{'d%d' % d:>7}" for d in DBG))
for i, o in enumerate(res[0]):
    if o["kind"] not in ("conv", "convgn"):
        continue
    print(f"{i:3d} {o['kind']:5} {o['M']:7d} {o['N']:5d} {o['K']:5d} {o['H']:3d} {o['ks']:2d} " +
          " ".join(f"{res[d][i]['ms']*1e3:7.1f}" for d in DBG))
