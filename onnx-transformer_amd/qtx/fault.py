"""Fault injection at the QuantLinear MatMuls — the reference's fault models on the qtx path.

The reference injects one fault per inference into a named MatMul of the exported encoder
or decoder graph (parallelized_inject_onnx_transformer.py:800-860 picks the target from
input/{encoder,decoder}/matmul_*.json, the fault model and the bit position; the fault is
applied by onnx_optimized_inference.py:59-204 with inject_utils/layers.py:48-84):

  INPUT / WEIGHT      one random element of the MatMul's int8 input (the output of its
                      activation quantizer) / int8 weight gets bit `b` flipped
                      (flip_int8_bit, layers.py:62-69); the perturbation propagates through
                      the MatMul (perturb_quantizer / perturb_matmul)
  INPUT16 / WEIGHT16  the same perturbation kept on a 16-wide window of output columns /
                      a window of up to 16 output rows (onnx_optimized_inference.py:121-186)
  RANDOM              one random element of the MatMul output replaced by a random fp32
                      (delta_init, layers.py:17-21); RANDOM_BITFLIP: one bit of it flipped

Here the fault is a ``qtx_fault`` handed to the fused HIP path (include/qtx.h): INPUT/WEIGHT
kinds correct the int32 accumulators exactly inside the GEMM, RANDOM kinds replace the
MatMul output before the bias.  Targets use the reference's MatMul numbering.
"""
from __future__ import annotations

import dataclasses
import re
import struct

import numpy as np

from . import _lib

KINDS = {"NONE": 0, "INPUT": 1, "WEIGHT": 2, "INPUT16": 3, "WEIGHT16": 4, "OUTPUT": 5,
         "RANDOM": 5, "RANDOM_BITFLIP": 5}
LIN = {"Q": 0, "K": 1, "V": 2, "QK": 3, "PV": 4, "O": 5, "FFN1": 6, "FFN2": 7, "CQ": 8, "CK": 9,
       "CV": 10, "CO": 11, "CQK": 12, "CPV": 13}
ATTN = ("QK", "PV", "CQK", "CPV")
_LIN_NAME = {v: k for k, v in LIN.items()}
# decoder layer: MatMul_{12 + 12 L + i}, i -> target (3/4 self QK^T / PV, 7/8 cross)
_DEC_LAYER_MM = {0: "Q", 1: "K", 2: "V", 3: "QK", 4: "PV", 5: "O", 6: "CQ", 7: "CQK", 8: "CPV",
                 9: "CO", 10: "FFN1", 11: "FFN2"}
_ENC_LAYER_MM = {0: "Q", 1: "K", 2: "V", 3: "QK", 4: "PV", 5: "O", 6: "FFN1", 7: "FFN2"}


def matmul_target(name: str, module: str, n_layers: int = 6):
    """Reference ONNX MatMul name -> (module id, layer, linear name).

    Encoder: MatMul_{8L+i}; decoder: MatMul_{2L} / MatMul_{2L+1} are the memory K / V
    projections of layer L, MatMul_{12+12L+i} the layer's own MatMuls.
    Attention MatMuls map to QK / PV (decoder cross: CQK / CPV)."""
    m = re.fullmatch(r"MatMul_(\d+)", name)
    if not m:
        raise ValueError(f"not a MatMul name: {name}")
    idx = int(m.group(1))
    if module.lower().startswith("enc"):
        layer, i = divmod(idx, 8)
        if layer >= n_layers or i not in _ENC_LAYER_MM:
            raise ValueError(f"{name}: not an encoder MatMul")
        return 0, layer, _ENC_LAYER_MM[i]
    if idx < 2 * n_layers:
        return 1, idx // 2, "CK" if idx % 2 == 0 else "CV"
    layer, i = divmod(idx - 2 * n_layers, 12)
    if layer >= n_layers or i not in _DEC_LAYER_MM:
        raise ValueError(f"{name}: not a decoder MatMul")
    return 1, layer, _DEC_LAYER_MM[i]


@dataclasses.dataclass
class Fault:
    """One injected fault (qtx_fault).  Rows index the module's flattened tokens."""
    kind: str                  # INPUT, WEIGHT, INPUT16, WEIGHT16, RANDOM, RANDOM_BITFLIP
    module: int                # 0 encoder, 1 decoder
    layer: int
    linear: str                # Q K V O FFN1 FFN2 CQ CK CV CO
    row: int = 0
    col: int = 0
    bit: int = 0
    win_start: int = 0
    win_len: int = 0
    value: float = 0.0

    def to_c(self) -> "_lib.Fault":
        return _lib.Fault(KINDS[self.kind], self.module, self.layer, LIN[self.linear],
                          int(self.row), int(self.col), int(self.win_start), int(self.win_len),
                          int(self.bit), float(self.value), 0)

    def as_dict(self):
        return dataclasses.asdict(self)


def linear_shape(linear: str, d_model=512, d_ff=2048):
    """(N, K) of the target QuantLinear."""
    return (d_ff if linear == "FFN1" else d_model, d_ff if linear == "FFN2" else d_model)


def random_attn_fault(rng, kind, module, layer, linear, B, Sq, Sk, H=8, bit=None,
                      golden_output=None):
    """Draw an attention-MatMul fault like the reference: uniform indices over the int
    tensor (q / P*127 input, k / v weight, [B, H, S, .]), INPUT16 a 16-aligned window of the
    output's last dim (keys for QK^T, head dims for PV), WEIGHT16 a 16-aligned start and
    1..15 query rows (onnx_optimized_inference.py:121-186).  golden_output for
    RANDOM_BITFLIP: the golden MatMul output [B, H, Sq, Sk|64]."""
    qk = linear in ("QK", "CQK")
    f = Fault(kind, module, layer, linear, bit=0 if bit is None else int(bit))
    b, h = int(rng.integers(B)), int(rng.integers(H))
    last = Sk if qk else 64
    if kind in ("INPUT", "INPUT16"):
        i = int(rng.integers(Sq))
        f.row = b * Sq + i
        f.col = h * 64 + int(rng.integers(64)) if qk else h * Sk + int(rng.integers(Sk))
        if kind == "INPUT16":
            f.win_start = 16 * int(rng.integers(max(last // 16, 1)))
            f.win_len = min(16, last - f.win_start)
    elif kind in ("WEIGHT", "WEIGHT16"):
        f.row = b * Sk + int(rng.integers(Sk))
        f.col = h * 64 + int(rng.integers(64))
        if kind == "WEIGHT16":
            f.win_start = 16 * int(rng.integers(max(Sq // 16, 1)))
            f.win_len = max(1, min(int(rng.integers(1, 16)), Sq - f.win_start))
    else:
        i, c = int(rng.integers(Sq)), int(rng.integers(last))
        f.row, f.col = b * Sq + i, h * last + c
        if kind == "RANDOM":
            v = struct.unpack("<f", struct.pack("<I", int(rng.integers(0, 2 ** 32))))[0]
        else:
            g = float(golden_output[b, h, i, c])
            u = struct.unpack("<I", struct.pack("<f", g))[0] ^ (1 << int(rng.integers(32)))
            v = struct.unpack("<f", struct.pack("<I", u))[0]
        f.value = 0.0 if np.isnan(v) else v
    return f


def random_fault(rng, kind, module, layer, linear, rows, bit=None, d_model=512, d_ff=2048,
                 golden_output=None):
    """Draw a fault the way the reference does: uniform indices over the target tensor
    (np.random.randint per dimension, layers.py:73 / onnx_optimized_inference.py:63), a
    16-aligned window for the *16 kinds (onnx_optimized_inference.py:123-131, 157-166:
    INPUT16 keeps 16 columns, WEIGHT16 a random 1..15 rows), a random fp32 for RANDOM
    (delta_init) and one flipped bit of the golden output for RANDOM_BITFLIP
    (float32_bit_flip; golden_output [rows, N] host array required)."""
    N, K = linear_shape(linear, d_model, d_ff)
    f = Fault(kind, module, layer, linear, bit=0 if bit is None else int(bit))
    if kind in ("INPUT", "INPUT16"):
        f.row, f.col = int(rng.integers(rows)), int(rng.integers(K))
        if kind == "INPUT16":
            f.win_start, f.win_len = 16 * int(rng.integers(max(N // 16, 1))), min(16, N)
    elif kind in ("WEIGHT", "WEIGHT16"):
        f.row, f.col = int(rng.integers(N)), int(rng.integers(K))
        if kind == "WEIGHT16":
            f.win_start = 16 * int(rng.integers(max(rows // 16, 1)))
            f.win_len = max(1, min(int(rng.integers(1, 16)), rows - f.win_start))
    else:
        f.row, f.col = int(rng.integers(rows)), int(rng.integers(N))
        if kind == "RANDOM":
            bits = int(rng.integers(0, 2 ** 32))
            v = struct.unpack("<f", struct.pack("<I", bits))[0]
            f.value = 0.0 if np.isnan(v) else v          # bin2fp32 maps NaN to 0
        else:
            g = float(golden_output[f.row, f.col])
            u = struct.unpack("<I", struct.pack("<f", g))[0] ^ (1 << int(rng.integers(32)))
            v = struct.unpack("<f", struct.pack("<I", u))[0]
            f.value = 0.0 if np.isnan(v) else v
    return f


def from_inject_parameters(p: dict, rows: int, rng=None, n_layers=6, golden_output=None,
                           attn_shape=None):
    """The reference's inject_parameters dict (parallelized_inject_onnx_transformer.py:
    837-858: inject_type, faulty_operation_name, targetted_module, faulty_bit_position)
    -> a Fault with indices drawn like the reference.  attn_shape (B, Sq, Sk) is needed for
    attention-MatMul targets."""
    rng = rng if rng is not None else np.random.default_rng()
    module, layer, linear = matmul_target(p["faulty_operation_name"], p["targetted_module"],
                                          n_layers)
    if linear in ATTN:
        B, Sq, Sk = attn_shape
        return random_attn_fault(rng, p["inject_type"], module, layer, linear, B, Sq, Sk,
                                 bit=p.get("faulty_bit_position"), golden_output=golden_output)
    return random_fault(rng, p["inject_type"], module, layer, linear, rows,
                        p.get("faulty_bit_position"), golden_output=golden_output)
