"""UNet architecture descriptions and the reference state_dict key surface.

The key names and shapes enumerated here are the ones the reference's
``torch.save(model.state_dict())`` produces, so checkpoints written by the
reference load unchanged (drop-in surface):

* DDPM UNet, ``Diffusion/Model.py:212-262`` (TimeEmbedding 15-42, ResBlock 167-200,
  AttnBlock 129-140, DownSample 96-104, UpSample 111-119).
* CFG UNet, ``DiffusionFreeGuidence/ModelCondition.py:164-203`` (TimeEmbedding table
  24-42, ConditionalEmbedding 49-58, DownSample 65-69, UpSample 76-80).

Nothing here computes; it only walks the constructor logic to name tensors.
"""
from __future__ import annotations

import dataclasses
from collections import OrderedDict
from typing import List, Sequence, Tuple

ARCH_DDPM = 0
ARCH_CFG = 1


@dataclasses.dataclass(frozen=True)
class UNetArch:
    """Constructor arguments of the reference UNets (``Model.py:213``,
    ``ModelCondition.py:165``)."""

    ch: int = 128
    ch_mult: Tuple[int, ...] = (1, 2, 3, 4)
    attn: Tuple[int, ...] = (2,)
    num_res_blocks: int = 2
    T: int = 1000
    img_size: int = 32
    kind: int = ARCH_DDPM
    num_labels: int = 10

    def __post_init__(self):
        object.__setattr__(self, "ch_mult", tuple(int(m) for m in self.ch_mult))
        object.__setattr__(self, "attn", tuple(int(a) for a in self.attn))
        assert all(i < len(self.ch_mult) for i in self.attn), "attn index out of bound"  # Model.py:215
        assert self.ch % 32 == 0, "GroupNorm(32, C) needs C % 32 == 0"

    @property
    def tdim(self) -> int:
        return self.ch * 4  # Model.py:216

    @property
    def cfg(self) -> bool:
        return self.kind == ARCH_CFG


# Arch A: config/config.yaml:25-29 (the CIFAR-10 DDPM UNet the metric is quoted on).
ARCH_A = UNetArch(ch=128, ch_mult=(1, 2, 3, 4), attn=(2,), num_res_blocks=2, T=1000, img_size=32)
# Arch C: MainCondition.py:10-13 (CFG UNet).
ARCH_C = UNetArch(ch=128, ch_mult=(1, 4, 8, 8, 4, 2), attn=(), num_res_blocks=2, T=1000,
                  img_size=32, kind=ARCH_CFG, num_labels=10)
# Tiny UNet used for golden vectors.
ARCH_TINY = UNetArch(ch=32, ch_mult=(1, 2), attn=(1,), num_res_blocks=1, T=1000, img_size=32)
ARCH_TINY_CFG = UNetArch(ch=32, ch_mult=(1, 2), attn=(), num_res_blocks=1, T=1000, img_size=32,
                         kind=ARCH_CFG, num_labels=10)


@dataclasses.dataclass
class BlockSpec:
    """One entry of downblocks / middleblocks / upblocks."""

    prefix: str
    kind: str  # "res", "down", "up"
    in_ch: int
    out_ch: int
    attn: bool = False


def block_specs(a: UNetArch) -> Tuple[List[BlockSpec], List[BlockSpec], List[BlockSpec]]:
    """Mirror of the module-list construction in ``Model.py:218-246`` /
    ``ModelCondition.py:171-197``."""
    down, mid, up = [], [], []
    chs = [a.ch]
    now = a.ch
    for i, mult in enumerate(a.ch_mult):
        out = a.ch * mult
        for _ in range(a.num_res_blocks):
            use_attn = (i in a.attn) if not a.cfg else True  # CFG ResBlock attn=True default (ModelCondition.py:122,177)
            down.append(BlockSpec(f"downblocks.{len(down)}", "res", now, out, use_attn))
            now = out
            chs.append(now)
        if i != len(a.ch_mult) - 1:
            down.append(BlockSpec(f"downblocks.{len(down)}", "down", now, now))
            chs.append(now)
    mid.append(BlockSpec("middleblocks.0", "res", now, now, True))
    mid.append(BlockSpec("middleblocks.1", "res", now, now, False))
    for i, mult in reversed(list(enumerate(a.ch_mult))):
        out = a.ch * mult
        for _ in range(a.num_res_blocks + 1):
            use_attn = (i in a.attn) if not a.cfg else False  # ModelCondition.py:193 attn=False
            up.append(BlockSpec(f"upblocks.{len(up)}", "res", chs.pop() + now, out, use_attn))
            now = out
        if i != 0:
            up.append(BlockSpec(f"upblocks.{len(up)}", "up", now, now))
    assert not chs
    return down, mid, up


def param_specs(a: UNetArch) -> "OrderedDict[str, Tuple[int, ...]]":
    """Every state_dict key the reference module registers, with its shape,
    in module registration order."""
    p: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
    d, td = a.ch, a.tdim

    def conv(name, cout, cin, k):
        p[name + ".weight"] = (cout, cin, k, k)
        p[name + ".bias"] = (cout,)

    def lin(name, cout, cin):
        p[name + ".weight"] = (cout, cin)
        p[name + ".bias"] = (cout,)

    def gn(name, c):
        p[name + ".weight"] = (c,)
        p[name + ".bias"] = (c,)

    if not a.cfg:
        p["time_embedding.freq_coeffs"] = (d // 2,)  # Model.py:34 buffer
        lin("time_embedding.timembedding.0", td, d)
        lin("time_embedding.timembedding.2", td, td)
    else:
        p["time_embedding.timembedding.0.weight"] = (a.T, d)  # nn.Embedding table, ModelCondition.py:38
        lin("time_embedding.timembedding.1", td, d)
        lin("time_embedding.timembedding.3", td, td)
        p["cond_embedding.condEmbedding.0.weight"] = (a.num_labels + 1, d)
        lin("cond_embedding.condEmbedding.1", td, d)
        lin("cond_embedding.condEmbedding.3", td, td)
    conv("head", d, 3, 3)
    down, mid, up = block_specs(a)
    for b in down + mid + up:
        if b.kind == "res":
            gn(b.prefix + ".block1.0", b.in_ch)
            conv(b.prefix + ".block1.2", b.out_ch, b.in_ch, 3)
            lin(b.prefix + ".temb_proj.1", b.out_ch, td)
            if a.cfg:
                lin(b.prefix + ".cond_proj.1", b.out_ch, td)
            gn(b.prefix + ".block2.0", b.out_ch)
            conv(b.prefix + ".block2.3", b.out_ch, b.out_ch, 3)
            if b.in_ch != b.out_ch:
                conv(b.prefix + ".shortcut", b.out_ch, b.in_ch, 1)
            if b.attn:
                gn(b.prefix + ".attn.group_norm", b.out_ch)
                for q in ("proj_q", "proj_k", "proj_v", "proj"):
                    conv(f"{b.prefix}.attn.{q}", b.out_ch, b.out_ch, 1)
        elif b.kind == "down":
            if not a.cfg:
                conv(b.prefix + ".main", b.in_ch, b.in_ch, 3)
            else:
                conv(b.prefix + ".c1", b.in_ch, b.in_ch, 3)
                conv(b.prefix + ".c2", b.in_ch, b.in_ch, 5)
        else:  # up
            if not a.cfg:
                conv(b.prefix + ".main", b.in_ch, b.in_ch, 3)
            else:
                conv(b.prefix + ".c", b.in_ch, b.in_ch, 3)
                # ConvTranspose2d weight is [Cin, Cout, k, k]
                p[b.prefix + ".t.weight"] = (b.in_ch, b.in_ch, 5, 5)
                p[b.prefix + ".t.bias"] = (b.in_ch,)
    last = up[-1].out_ch
    gn("tail.0", last)
    conv("tail.2", 3, last, 3)
    return p


def flops_per_image(a: UNetArch) -> float:
    """Algorithmic FLOPs (2 per MAC) of one UNet forward on one image, counting
    convolutions, attention matmuls and Linears (the FlopCounterMode convention
    SURVEY.md 8(d) quotes: 14.88 GFLOP for Arch A at 32 px)."""
    H = a.img_size
    fl = 0.0
    td = a.tdim
    fl += 2 * (a.ch * td + td * td)
    fl += 2 * H * H * 3 * a.ch * 9  # head
    down, mid, up = block_specs(a)
    res = H
    for b in down + mid + up:
        if b.kind == "res":
            fl += 2 * res * res * b.in_ch * b.out_ch * 9
            fl += 2 * res * res * b.out_ch * b.out_ch * 9
            fl += 2 * td * b.out_ch * (2 if a.cfg else 1)
            if b.in_ch != b.out_ch:
                fl += 2 * res * res * b.in_ch * b.out_ch
            if b.attn:
                S, C = res * res, b.out_ch
                fl += 4 * 2 * S * C * C + 2 * 2 * S * S * C
        elif b.kind == "down":
            res //= 2
            fl += 2 * res * res * b.in_ch * b.in_ch * (9 + (25 if a.cfg else 0))
        else:
            res *= 2
            fl += 2 * res * res * b.in_ch * b.in_ch * 9
            if a.cfg:
                fl += 2 * (res // 2) ** 2 * b.in_ch * b.in_ch * 25
    fl += 2 * H * H * up[-1].out_ch * 3 * 9  # tail
    return fl
