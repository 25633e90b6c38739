"""CPU-side checks of the boundary: the C-ABI library loads and exports every
symbol include/itsd.h declares; host-side helpers behave (no GPU compute here)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import ROOT
import itsd
from itsd import runtime as rt
from itsd.arch import ARCH_A, ARCH_C, ARCH_TINY, flops_per_image, param_specs
from itsd.diffusion import reference_noise_plan
from itsd.weights import check_state_dict, synthetic_state_dict


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "itsd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(itsd_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    if not os.path.exists(rt.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    L = ctypes.CDLL(rt.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 9
    for s in syms:
        assert hasattr(L, s), f"missing export {s}"
    assert set(syms) == set(rt.EXPORTS), "runtime.py bindings out of sync with include/itsd.h"
    assert L.itsd_version() == 1


def test_param_specs_match_reference_key_counts():
    # Arch A has 333 keys, Arch C 614
    assert len(param_specs(ARCH_A)) == 333
    assert len(param_specs(ARCH_C)) == 614


def test_flops_archA():
    # 14.882 GFLOP per 32px image forward (FlopCounterMode)
    assert abs(flops_per_image(ARCH_A) / 1e9 - 14.882) < 0.01


def test_state_dict_checks():
    sd = synthetic_state_dict(ARCH_TINY, 0)
    check_state_dict(ARCH_TINY, sd)
    bad = dict(sd)
    bad.pop("head.weight")
    with pytest.raises(KeyError):
        check_state_dict(ARCH_TINY, bad)
    bad = dict(sd)
    bad["head.bias"] = torch.zeros(3)
    with pytest.raises(ValueError):
        check_state_dict(ARCH_TINY, bad)


def test_reference_noise_plan_order():
    torch.manual_seed(3)
    x_T, noise = reference_noise_plan((1, 3, 4, 4), T=4, n_runs=2)
    torch.manual_seed(3)
    seq = [torch.randn(1, 3, 4, 4) for _ in range(2 * 4)]
    # run 0: x_T, z(t=3), z(2), z(1); run 1: x_T, z(3), z(2), z(1)
    assert torch.equal(x_T[0], seq[0]) and torch.equal(x_T[1], seq[4])
    for run in range(2):
        for k, t in enumerate([3, 2, 1]):
            assert torch.equal(noise[t, run], seq[4 * run + 1 + k][0])
    assert torch.count_nonzero(noise[0]) == 0


def test_conv_tile_options():
    """The conv tile switches (itsd_set_option) accept 0 off / 1 auto / 2 whenever eligible and
    reject other values; the switches of kernels that only diagnostic builds contain (the
    superseded 256-pixel generations, conv_pipe_wide, the compile-time ablations) fail loudly in
    the shipped library; the removed generations are refused. Host-side only (no device call)."""
    if not os.path.exists(rt.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    for key, default in (("gn_wide", 1), ("small_conv", 1)):
        for v in (0, 1, 2):
            rt.set_option(key, v)
        with pytest.raises(rt.ItsdError):
            rt.set_option(key, 3)
        rt.set_option(key, default)
    # measured-and-dropped paths (removed in rounds 4-5): their switches are unknown keys or refused values
    for key, val in (("conv_wide", 0), ("gn_reg", 4), ("tail_px", 64), ("p4_m16", 1), ("small_korder", 1)):
        with pytest.raises(rt.ItsdError, match="unknown option"):
            rt.set_option(key, val)
    for key, val, default in (("attn_fuse", 2, 1), ("attn_s1", 2, 1), ("p4_w", 15, 7), ("conv_variant", 3, 2), ("conv_variant", 0, 2)):
        with pytest.raises(rt.ItsdError):
            rt.set_option(key, val)
        rt.set_option(key, default)
    for v in (0, 2, 1):  # 96-cout 8x8 tiles: off / always / auto (shipped)
        rt.set_option("p4_c96", v)
    with pytest.raises(rt.ItsdError):
        rt.set_option("p4_c96", 3)
    for v in (0, 2, 1):  # 1x1 shortcuts as K slices of their block2 p5 conv: off / always / auto (shipped)
        rt.set_option("p5_sc", v)
    with pytest.raises(rt.ItsdError):
        rt.set_option("p5_sc", 3)
    rt.set_option("spin_bound", 0)  # diagnostic (fail-loud hand-off test), any bound >= 0
    rt.set_option("spin_bound", 1 << 22)
    with pytest.raises(rt.ItsdError):
        rt.set_option("spin_bound", -1)
    # (round 6) measurement switches are diagnostic-build only: the shipped ABI refuses them
    for key, val in (("conv_dbg", 1), ("conv_dbg", 0), ("attn_cs", 2), ("attn_aq", 32), ("p4_xcd", 1),
                     ("small_minks", 2), ("splitk", 2), ("conv1x1", 2), ("p5_c64", 2)):
        with pytest.raises(rt.ItsdError, match="diagnostic build"):
            rt.set_option(key, val)
    for key, val in (("splitk", 0), ("splitk", 1), ("conv1x1", 0), ("conv1x1", 1)):  # their shipped values stay
        rt.set_option(key, val)
    # a refused value leaves the previous setting in place (validated before it is stored)
    for v in (0, 2, 1):
        rt.set_option("p5_dist", v)
    assert rt.lib().itsd_set_option(b"p5_dist", 3) != 0
    for v in (0, 1):  # (round 6) p5's two-slice combine: both slices publish / only the first (shipped)
        rt.set_option("p5_pub", v)
    assert rt.lib().itsd_set_option(b"p5_pub", 2) != 0
    for v in (0, 1, 2, 3):  # (round 6) p5's split-K exchange through one XCD's L2: off / shared combine / every form / shipped
        rt.set_option("p5_xl", v)
    assert rt.lib().itsd_set_option(b"p5_xl", 4) != 0
    for v in (0, 1):  # (round 6) conv_small's fused consumer GroupNorm: off / on (shipped)
        rt.set_option("small_gn", v)
    assert rt.lib().itsd_set_option(b"small_gn", 2) != 0


def test_shipped_library_holds_only_product_kernels():
    """measurement scaffolding stays out of the shipped .so -- no superseded fused-conv
    kernel (wide / reg / ws / pws), no conv_pipe_wide, no stamps symbol (tools/build_diag.sh builds
    them into build_diag/ instead)."""
    if not os.path.exists(rt.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    blob = open(rt.LIB_PATH, "rb").read()
    for name in (b"conv3x3_gn_wide_kernel", b"conv3x3_gn_reg_kernel", b"conv3x3_gn_ws_kernel",
                 b"conv3x3_gn_pws_kernel", b"conv_pipe_wide", b"itsd_debug_stamps",
                 # round 5: the dropped 16x16x32 p4 form, p4 at 64x64, the 4-image AttnBlock, 3/4-stage pipes
                 b"conv3x3_gn_p4_kernelILi32ELi0ELb1", b"conv3x3_gn_p4_kernelILi64", b"attn_block_kernelILi512ELi4",
                 b"conv_pipeItLi3", b"conv_pipeItLi4", b"tail_mfma_kernelILi64"):
        assert name not in blob, name
    assert b"conv3x3_gn_p4_kernel" in blob
