"""ctypes binding of libitsd_hip.so (the C ABI in include/itsd.h).

The library is the product: there is no CPU or PyTorch fallback. If the shared
object is missing or fails to load, every entry point raises.
Tensors cross the boundary as raw device pointers (``tensor.data_ptr()``) plus the
current ROCm stream handle; ctypes releases the GIL for the call.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Sequence

import torch

from .arch import ARCH_CFG, ARCH_DDPM, UNetArch

_HERE = os.path.dirname(os.path.abspath(__file__))
# ITSD_LIB: an alternative build of the same library (diagnostic A/B builds under build_diag/)
LIB_PATH = os.environ.get("ITSD_LIB") or os.path.join(_HERE, "libitsd_hip.so")

ITSD_OK, ITSD_ERR_INVALID, ITSD_ERR_HIP, ITSD_ERR_WEIGHTS, ITSD_ERR_NAN, ITSD_ERR_OOM, ITSD_ERR_HANDOFF = range(7)
PREC_FP32, PREC_BF16 = 0, 1
VERIFY_ORACLE, VERIFY_SELFSUP, VERIFY_AESTHETIC, VERIFY_MEAN = 0, 1, 2, 3
RUN_GRAPH, RUN_CLIP, RUN_SYNC = 1, 2, 4


class ItsdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[itsd error {code}] {msg}")
        self.code = code


class UNetDesc(ctypes.Structure):
    _fields_ = [("arch", ctypes.c_int32), ("T", ctypes.c_int32), ("ch", ctypes.c_int32),
                ("n_mult", ctypes.c_int32), ("ch_mult", ctypes.c_int32 * 8), ("n_attn", ctypes.c_int32),
                ("attn", ctypes.c_int32 * 8), ("num_res_blocks", ctypes.c_int32), ("img_size", ctypes.c_int32),
                ("num_labels", ctypes.c_int32), ("max_batch", ctypes.c_int32), ("precision", ctypes.c_int32)]


class TensorView(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("numel", ctypes.c_int64)]


_lib = None

_SIGS = {
    "itsd_unet_create": [ctypes.POINTER(UNetDesc), ctypes.POINTER(TensorView), ctypes.c_int, ctypes.c_int,
                         ctypes.POINTER(ctypes.c_void_p)],
    "itsd_unet_destroy": [ctypes.c_void_p],
    "itsd_unet_forward": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_int, ctypes.c_void_p],
    "itsd_unet_representation": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p],
    "itsd_set_schedule": [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_float],
    "itsd_sampler_run": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                         ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p],
    "itsd_noise": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64,
                   ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p],
    "itsd_verify": [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                    ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p],
    "itsd_verify_paired": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p, ctypes.c_void_p],
    "itsd_attention": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                       ctypes.c_int, ctypes.c_void_p],
    "itsd_profile_forward": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double), ctypes.c_void_p],
    "itsd_profile_op": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                        ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_void_p],
    "itsd_profile_ops": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.POINTER(ctypes.c_int), ctypes.c_void_p],
    "itsd_set_option": [ctypes.c_char_p, ctypes.c_int],
    "itsd_calibrate": [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_void_p],
    "itsd_unet_query": [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)],
    "itsd_kernel_name": [ctypes.c_int],
    "itsd_last_error": [],
    "itsd_version": [],
}

EXPORTS = tuple(_SIGS)


def lib():
    """Load libitsd_hip.so (raises if absent: the HIP path is the only path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ItsdError(ITSD_ERR_INVALID, f"{LIB_PATH} is not built; run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        shipped = os.path.abspath(LIB_PATH) == os.path.join(_HERE, "libitsd_hip.so")
        for name, args in _SIGS.items():
            if not shipped and not hasattr(L, name):
                continue  # (an older build loaded for an A/B measurement: entry points it predates are absent)
            f = getattr(L, name)
            f.argtypes = args
            f.restype = ctypes.c_char_p if name in ("itsd_last_error", "itsd_kernel_name") else ctypes.c_int
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != ITSD_OK:
        msg = lib().itsd_last_error().decode(errors="replace")
        if rc == ITSD_ERR_NAN:
            raise AssertionError(msg)  # Diffusion.py:100 assert semantics
        raise ItsdError(rc, msg)


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


class NativeUNet:
    """Owns one itsd_unet handle (weights repacked on the device, workspace for max_batch)."""

    def __init__(self, arch: UNetArch, state_dict: Dict[str, torch.Tensor], max_batch: int, precision: int,
                 device: int = 0):
        L = lib()
        d = UNetDesc()
        d.arch = ARCH_CFG if arch.cfg else ARCH_DDPM
        d.T = arch.T
        d.ch = arch.ch
        d.n_mult = len(arch.ch_mult)
        for i, m in enumerate(arch.ch_mult):
            d.ch_mult[i] = m
        d.n_attn = len(arch.attn)
        for i, m in enumerate(arch.attn):
            d.attn[i] = m
        d.num_res_blocks = arch.num_res_blocks
        d.img_size = arch.img_size
        d.num_labels = arch.num_labels
        d.max_batch = int(max_batch)
        d.precision = int(precision)
        keep = []
        views = (TensorView * len(state_dict))()
        for i, (k, v) in enumerate(state_dict.items()):
            hv = v.detach().to("cpu", torch.float32).contiguous()
            keep.append(hv)
            views[i].name = k.encode()
            views[i].data = hv.data_ptr()
            views[i].numel = hv.numel()
        h = ctypes.c_void_p()
        check(L.itsd_unet_create(ctypes.byref(d), views, len(state_dict), int(device), ctypes.byref(h)))
        self.h = h
        self.arch = arch
        self.max_batch = int(max_batch)
        self.precision = int(precision)
        self.device = int(device)
        self.T_sched = 0

    def close(self):
        if getattr(self, "h", None):
            lib().itsd_unet_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def forward(self, x: torch.Tensor, t: torch.Tensor, labels: Optional[torch.Tensor], eps: torch.Tensor) -> None:
        check(lib().itsd_unet_forward(self.h, x.data_ptr(), t.data_ptr(), _ptr(labels), eps.data_ptr(),
                                      x.shape[0], stream_ptr(x.device)))

    def representation(self, n: int, channels: int, hw: int, device) -> torch.Tensor:
        """The pre-tail activation of the last forward as NCHW fp32 [n, channels, hw, hw]."""
        out = torch.empty(n, channels, hw, hw, dtype=torch.float32, device=device)
        check(lib().itsd_unet_representation(self.h, out.data_ptr(), int(n), stream_ptr(out.device)))
        return out

    def set_schedule(self, coeff1: torch.Tensor, coeff2: torch.Tensor, sqrt_var: torch.Tensor, w: float = 0.0):
        c1 = coeff1.detach().cpu().float().contiguous()
        c2 = coeff2.detach().cpu().float().contiguous()
        sv = sqrt_var.detach().cpu().float().contiguous()
        check(lib().itsd_set_schedule(self.h, c1.numel(), c1.data_ptr(), c2.data_ptr(), sv.data_ptr(), float(w)))
        self.T_sched = c1.numel()

    def run(self, x: torch.Tensor, t_begin: int, t_end: int, seed: int, noise: Optional[torch.Tensor] = None,
            labels: Optional[torch.Tensor] = None, noise_offset: int = 0, graph: bool = True, clip: bool = True,
            sync: bool = True) -> None:
        flags = (RUN_GRAPH if graph else 0) | (RUN_CLIP if clip else 0) | (RUN_SYNC if sync else 0)
        check(lib().itsd_sampler_run(self.h, x.data_ptr(), _ptr(labels), x.shape[0], int(t_begin), int(t_end),
                                     int(seed) & ((1 << 64) - 1), int(noise_offset), _ptr(noise), flags,
                                     stream_ptr(x.device)))

    def query(self, key: str) -> int:
        """itsd_unet_query: "graph_captures", "max_batch", "T_sched", "ws_bytes", "ops"."""
        v = ctypes.c_int64()
        check(lib().itsd_unet_query(self.h, key.encode(), ctypes.byref(v)))
        return int(v.value)

    def profile_forward(self, x: torch.Tensor, t: torch.Tensor):
        cm, cf, tm = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        cl = ctypes.c_int()
        check(lib().itsd_profile_forward(self.h, x.data_ptr(), t.data_ptr(), x.shape[0], ctypes.byref(cm),
                                         ctypes.byref(cf), ctypes.byref(cl), ctypes.byref(tm), stream_ptr(x.device)))
        return {"conv_ms": cm.value, "conv_flops": cf.value, "conv_launches": cl.value, "total_ms": tm.value}

    def profile_op(self, x: torch.Tensor, t: torch.Tensor, op_index: int, reps: int = 10) -> float:
        """Steady-state ms of program op `op_index` (profile_ops numbering), `reps` back-to-back launches."""
        ms = ctypes.c_double()
        check(lib().itsd_profile_op(self.h, x.data_ptr(), t.data_ptr(), x.shape[0], int(op_index), int(reps),
                                    ctypes.byref(ms), stream_ptr(x.device)))
        return ms.value

    def profile_ops(self, x: torch.Tensor, t: torch.Tensor, max_ops: int = 512):
        import numpy as np

        kinds = np.zeros(max_ops, np.int32)
        ms = np.zeros(max_ops, np.float64)
        fl = np.zeros(max_ops, np.float64)
        sh = np.zeros((max_ops, 8), np.int32)
        n = ctypes.c_int()
        check(lib().itsd_profile_ops(self.h, x.data_ptr(), t.data_ptr(), x.shape[0], max_ops,
                                     kinds.ctypes.data, ms.ctypes.data, fl.ctypes.data, sh.ctypes.data,
                                     ctypes.byref(n), stream_ptr(x.device)))
        k = n.value
        names = {0: "gn", 1: "conv", 2: "attn", 3: "gncoef", 4: "convgn", 5: "convgnw", 6: "convgnw4", 7: "attnblock",
                 -1: "head", -2: "tail"}
        L = lib()

        def decode(v: int):  # (kernel id << 8) | op class as a signed byte
            base = v & 0xFF
            base = base - 256 if base >= 128 else base
            return names.get(base, str(base)), L.itsd_kernel_name(v >> 8).decode()

        dec = [decode(int(kinds[i])) for i in range(k)]
        return [{"kind": dec[i][0], "kernel": dec[i][1], "ms": float(ms[i]), "flops": float(fl[i]),
                 "M": int(sh[i, 0]), "N": int(sh[i, 1]), "K": int(sh[i, 2]), "H": int(sh[i, 3]),
                 "ks": int(sh[i, 4]), "stride_up": int(sh[i, 5]), "op": int(sh[i, 6]),
                 "resid": bool(sh[i, 7] & 1), "stats_out": bool(sh[i, 7] & 2), "gn_in": bool(sh[i, 7] & 4),
                 "sc_cin": int(sh[i, 7]) >> 8}
                for i in range(k)]


def noise(out: torch.Tensor, n_cand: int, seed: int, stream_id: int, cand_offset: int = 0,
          pivot: Optional[torch.Tensor] = None, scale: float = 1.0) -> torch.Tensor:
    per = out.numel() // max(1, n_cand)
    check(lib().itsd_noise(out.data_ptr(), _ptr(pivot), int(n_cand), int(per), float(scale),
                           int(seed) & ((1 << 64) - 1), int(stream_id) & 0xFFFFFFFF, int(cand_offset),
                           stream_ptr(out.device)))
    return out


CALIB_MFMA_BF16, CALIB_HBM_COPY, CALIB_MFMA_BF16_16X16 = 0, 1, 2


def calibrate(what: int) -> float:
    """On-box achievable peak: CALIB_MFMA_BF16 (32x32x16) / CALIB_MFMA_BF16_16X16 -> TFLOP/s, CALIB_HBM_COPY -> GB/s
    (itsd_calibrate)."""
    v = ctypes.c_double(0.0)
    check(lib().itsd_calibrate(int(what), ctypes.byref(v), stream_ptr()))
    return v.value


def set_option(key: str, value: int) -> None:
    check(lib().itsd_set_option(key.encode(), int(value)))


def verify(kind: int, images: torch.Tensor, n_cand: int) -> torch.Tensor:
    """Per-candidate scores (float64, on the images' device)."""
    assert images.dtype == torch.float32 and images.is_contiguous() and images.is_cuda
    N, C, H, W = images.shape
    assert N % n_cand == 0, "images must split evenly into candidates"
    scores = torch.empty(n_cand, dtype=torch.float64, device=images.device)
    check(lib().itsd_verify(int(kind), images.data_ptr(), int(n_cand), N // n_cand, C, H, W, scores.data_ptr(),
                            stream_ptr(images.device)))
    return scores


def verify_paired(images: torch.Tensor, ref_features: torch.Tensor) -> torch.Tensor:
    """Per-image cosine of the 8x8-pooled features with reference feature rows (float64)."""
    assert images.dtype == torch.float32 and images.is_contiguous() and images.is_cuda
    N, C, H, W = images.shape
    ref = ref_features.to(images.device, torch.float32).contiguous()
    assert ref.shape == (N, C * 64), f"reference features must be [{N}, {C * 64}]"
    scores = torch.empty(N, dtype=torch.float64, device=images.device)
    check(lib().itsd_verify_paired(images.data_ptr(), ref.data_ptr(), int(N), C, H, W, scores.data_ptr(),
                                   stream_ptr(images.device)))
    return scores


def attention(qkv: torch.Tensor, vt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """AttnBlock core (Model.py:152-161) on qkv [n][S][3C]; bf16 inputs take the MFMA
    kernels and need vt = V channel-major [n][C][S]. Returns out [n][S][C]."""
    assert qkv.is_cuda and qkv.is_contiguous() and qkv.dim() == 3 and qkv.shape[2] % 3 == 0
    n, S, C3 = qkv.shape
    C = C3 // 3
    prec = PREC_BF16 if qkv.dtype == torch.bfloat16 else PREC_FP32
    assert prec == PREC_BF16 or qkv.dtype == torch.float32
    if vt is not None:
        assert vt.dtype == qkv.dtype and vt.is_contiguous() and tuple(vt.shape) == (n, C, S)
    out = torch.empty(n, S, C, dtype=qkv.dtype, device=qkv.device)
    check(lib().itsd_attention(qkv.data_ptr(), _ptr(vt), out.data_ptr(), n, S, C, prec, stream_ptr(qkv.device)))
    return out
