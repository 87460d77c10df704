"""ctypes binding of libqtx.so (include/qtx.h).

Loading fails loudly: there is no CPU fallback in the product path.  torch is used only
for device memory and the current HIP stream (plumbing, not compute).
"""
from __future__ import annotations

import ctypes as C
import os
import re

from . import _build

_lib = None


class QtxError(RuntimeError):
    """Raised for a non-zero qtx_status (the reference raises on bad feeds/shapes too)."""

    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed (status {code}): {msg}")
        self.code = code


class QtxConfig(C.Structure):
    _fields_ = [(n, C.c_int32) for n in
                ("src_vocab", "tgt_vocab", "n_layers", "d_model", "d_ff", "n_heads",
                 "max_len", "weight_bits")]


P = C.c_void_p
I32, I64, SZ, F32 = C.c_int32, C.c_int64, C.c_size_t, C.c_float


class RowGemm(C.Structure):
    """struct qtx_row_gemm (include/qtx.h)."""
    _fields_ = [("A", P), ("sa", P), ("W", P), ("sw", P), ("bias", P),
                ("M", I32), ("N", I32), ("K", I32), ("epi", I32),
                ("out8", P), ("ldo8", I64), ("o8_ts", I64), ("os", P), ("os_ts", I64),
                ("res", P), ("xout", P), ("ln_a", P), ("ln_b", P),
                ("lnq", P), ("lns", P), ("lnout", P),
                ("pmax_out", P), ("pmax_in", P), ("pmax_n", I32), ("kp", I32), ("status", P),
                ("part", P), ("ksplit", I32)]

class FfnRows(C.Structure):
    """struct qtx_ffn_args (include/qtx.h)."""
    _fields_ = [("A", P), ("sa", P), ("wf", P), ("sw1", P), ("b1", P), ("sw2", P), ("b2", P),
                ("x", P), ("ln_a", P), ("ln_b", P), ("lnq", P), ("lns", P), ("lnout", P),
                ("M", I32), ("F", I32)]


class Fault(C.Structure):
    """struct qtx_fault (include/qtx.h)."""
    _fields_ = [("kind", I32), ("module", I32), ("layer", I32), ("linear", I32),
                ("row", I64), ("col", I64), ("win_start", I64), ("win_len", I32),
                ("bit", I32), ("value", F32), ("reserved", I32)]


FP = C.POINTER(Fault)

# name -> (restype, argtypes); must match include/qtx.h
SIGNATURES = {
    "qtx_last_error": (C.c_char_p, []),
    "qtx_version": (C.c_char_p, []),
    "qtx_model_tensor_count": (I32, [C.POINTER(QtxConfig)]),
    "qtx_model_create": (I32, [C.POINTER(QtxConfig), C.POINTER(P), I32, P, P, C.POINTER(P)]),
    "qtx_model_destroy": (I32, [P]),
    "qtx_model_device_bytes": (SZ, [P]),
    "qtx_model_linear": (I32, [P, I32, I32, I32, C.POINTER(P), C.POINTER(P), C.POINTER(P),
                               C.POINTER(I32), C.POINTER(I32)]),
    "qtx_model_norm": (I32, [P, I32, I32, I32, C.POINTER(P), C.POINTER(P)]),
    "qtx_encoder_workspace_size": (SZ, [P, I32, I32]),
    "qtx_decoder_workspace_size": (SZ, [P, I32, I32, I32]),
    "qtx_greedy_workspace_size": (SZ, [P, I32, I32, I32]),
    "qtx_encoder_forward": (I32, [P, P, P, I32, I32, P, P, SZ, P]),
    "qtx_decoder_forward": (I32, [P, P, P, P, P, I32, I32, I32, I32, P, P, SZ, P]),
    "qtx_greedy_decode": (I32, [P, P, P, I32, I32, I32, I64, P, P, SZ, P]),
    "qtx_encoder_forward_fault": (I32, [P, P, P, I32, I32, P, P, SZ, FP, P]),
    "qtx_decoder_forward_fault": (I32, [P, P, P, P, P, I32, I32, I32, I32, P, P, SZ, FP, P]),
    "qtx_greedy_decode_fault": (I32, [P, P, P, I32, I32, I32, I64, P, P, SZ, FP, P]),
    "qtx_embed": (I32, [P, I32, P, I32, I32, I32, P, P]),
    "qtx_generator": (I32, [P, P, I32, P, P, P, SZ, P]),
    "qtx_row_quant": (I32, [P, I32, I32, F32, P, P, P]),
    "qtx_layernorm_quant": (I32, [P, P, P, I32, I32, P, P, P, P]),
    "qtx_linear_i8": (I32, [P, P, P, P, P, I32, I32, I32, I32, I32, P, P, P]),
    "qtx_linear_rows": (I32, [C.POINTER(RowGemm), P]),
    "qtx_pack_w_kp": (I32, [P, I32, I32, P, P]),
    "qtx_pack_w_ws": (I32, [P, I32, I32, P, P]),
    "qtx_ffn_rows": (I32, [C.POINTER(FfnRows), P]),
    "qtx_pack_ffn": (I32, [P, P, I32, P, P]),
    "qtx_pack_int4": (I32, [P, I32, I32, P, P]),
    "qtx_attention_i8": (I32, [P, P, P, P, P, P, P, I64, I64, I32, I32, I32, I32, P, I32, P]),
    "qtx_attention_trace": (I32, [P, P, P, P, P, P, P, I64, I64, I32, I32, I32, I32, P, P, P, I32, P]),
    "qtx_attention_i8_quant": (I32, [P, P, P, P, P, P, P, I32, I32, P, P, P]),
    "qtx_skinny_linear": (I32, [I32, P, P, P, I64, P, P, P, I32, P, P, P, I32, I32, I32, I32,
                                I32, P, P, P, P]),
    "qtx_decode_attention": (I32, [I32, P, I64, P, P, P, P, I32, P, I32, P, I32, P, P, P]),
    "qtx_decode_argmax_embed": (I32, [P, P, I32, P, I64, P, P, P]),
    "qtx_debug_nop": (I32, [P]),
    "qtx_debug_reload_knobs": (I32, []),
    "qtx_model_check": (I32, [P, P]),
}


def header_symbols(path=None) -> list[str]:
    """Function names declared in include/qtx.h (used by the ABI test)."""
    path = path or os.path.join(_build.REPO, "include", "qtx.h")
    text = open(path).read()
    return sorted(set(re.findall(r"\b(qtx_[a-z0-9_]+)\s*\(", text)))


def lib(build: bool = True):
    """Load (building first if sources changed) libqtx.so; raises if impossible."""
    global _lib
    if _lib is not None:
        return _lib
    path = _build.build() if build else _build.LIB
    if os.environ.get("QTX_LIB_PATH"):        # diagnostic builds (tools/kernel_bench.py)
        path = os.environ["QTX_LIB_PATH"]
    if not os.path.exists(path):
        raise RuntimeError(f"libqtx.so missing at {path}; run __graft_entry__.build()")
    L = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    _lib = L
    return L


def call(name, *args):
    """Call an int32-status entry point and raise QtxError on failure."""
    L = lib()
    rc = getattr(L, name)(*args)
    if rc != 0:
        raise QtxError(name, rc, L.qtx_last_error().decode(errors="replace"))
    return rc


def reload_knobs():
    """Re-read the library's environment switches (qtx_debug_reload_knobs): they are read
    once per process otherwise (csrc/qtx_knobs.h)."""
    lib().qtx_debug_reload_knobs()
