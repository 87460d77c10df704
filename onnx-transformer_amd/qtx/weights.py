"""Model description, synthetic weights and the canonical tensor order of the C-ABI.

The state-dict key names are exactly those of the reference's ``make_model``
(``/root/reference/model.py:15-37``), so a real ``checkpoint/*.pt`` (absent from the
reference snapshot) loads through :func:`load_checkpoint` unchanged.

Synthetic weights are drawn from ``numpy.random.default_rng(seed)``:

* every tensor with dim > 1 (linears, embedding LUTs, generator) is Xavier-uniform,
  bound ``sqrt(6 / (fan_in + fan_out))`` — the init of ``model.py:34-36``;
* linear biases are ``U(+-1/sqrt(fan_in))`` (``nn.Linear``'s default);
* LayerNorm ``a_2 = 1``, ``b_2 = 0`` (``layer_norm.py:8-9``) unless ``ln_random`` asks
  for ``a_2 ~ U(0.5, 1.5)``, ``b_2 ~ U(-0.1, 0.1)`` so that tests exercise both terms;
* the positional-encoding buffer is built by :func:`positional_table` (torch, so that
  it is bit-identical to ``positional_encodings.py:14-20``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

DEFAULT_SEED = 20241223

BOS, EOS, PAD, UNK = 0, 1, 2, 3  # reference/onnx_reference_inference.py:204,249-250


@dataclass(frozen=True)
class ModelConfig:
    """Hyper-parameters of ``make_model`` (``model.py:15-16``) and the IWSLT14 vocab."""

    src_vocab: int = 5337
    tgt_vocab: int = 4444
    n_layers: int = 6
    d_model: int = 512
    d_ff: int = 2048
    n_heads: int = 8
    max_len: int = 5000  # positional_encodings.py:9
    weight_bits: int = 8  # 8 = W8A8 (quant_linear.py:114-116); 4 = packed int4 weights

    @property
    def d_k(self) -> int:
        return self.d_model // self.n_heads


# --------------------------------------------------------------------------------------
# Canonical linear order.  One "linear" = (weight [N, K], bias [N]).  The C-ABI's
# qtx_model_create() receives the fp32 tensors in exactly this order.
# --------------------------------------------------------------------------------------

def linear_names(cfg: ModelConfig = ModelConfig()) -> list[str]:
    """Prefixes of every W8A8 linear, in the order the C-ABI expects them."""
    names = []
    for L in range(cfg.n_layers):
        p = f"encoder.layers.{L}"
        names += [f"{p}.self_attn.linears.{i}" for i in range(4)]
        names += [f"{p}.feed_forward.w_1", f"{p}.feed_forward.w_2"]
    for L in range(cfg.n_layers):
        p = f"decoder.layers.{L}"
        names += [f"{p}.self_attn.linears.{i}" for i in range(4)]
        names += [f"{p}.src_attn.linears.{i}" for i in range(4)]
        names += [f"{p}.feed_forward.w_1", f"{p}.feed_forward.w_2"]
    return names


def norm_names(cfg: ModelConfig = ModelConfig()) -> list[str]:
    """Prefixes of every LayerNorm (a_2, b_2), in C-ABI order."""
    names = []
    for L in range(cfg.n_layers):
        names += [f"encoder.layers.{L}.sublayer.{i}.norm" for i in range(2)]
    names.append("encoder.norm")
    for L in range(cfg.n_layers):
        names += [f"decoder.layers.{L}.sublayer.{i}.norm" for i in range(3)]
    names.append("decoder.norm")
    return names


def tensor_order(cfg: ModelConfig = ModelConfig()) -> list[str]:
    """Full list of state-dict keys handed to ``qtx_model_create`` (see include/qtx.h)."""
    keys = []
    for n in linear_names(cfg):
        keys += [f"{n}.weight", f"{n}.bias"]
    for n in norm_names(cfg):
        keys += [f"{n}.a_2", f"{n}.b_2"]
    keys += ["src_embed.0.lut.weight", "tgt_embed.0.lut.weight",
             "generator.proj.weight", "generator.proj.bias"]
    return keys


def _linear_shape(name: str, cfg: ModelConfig) -> tuple[int, int]:
    if name.endswith("w_1"):
        return cfg.d_ff, cfg.d_model
    if name.endswith("w_2"):
        return cfg.d_model, cfg.d_ff
    return cfg.d_model, cfg.d_model


def positional_table(d_model: int = 512, max_len: int = 5000):
    """Sinusoidal table, same torch float32 ops as positional_encodings.py:14-20.

    Computed with torch (not numpy) so that sin/cos round exactly as the reference's.
    Returns a float32 numpy array [max_len, d_model].
    """
    import torch

    pe = torch.zeros(max_len, d_model)
    position = torch.arange(0.0, max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0.0, d_model, 2) * -(math.log(10000.0) / d_model))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe.numpy().astype(np.float32)


def synthetic_state_dict(seed: int = DEFAULT_SEED, cfg: ModelConfig = ModelConfig(),
                         ln_random: bool = False, with_pe: bool = True) -> dict:
    """Deterministic synthetic weights with the reference's key names (numpy float32)."""
    rng = np.random.default_rng(seed)
    sd: dict[str, np.ndarray] = {}

    def xavier(n_out, n_in):
        a = math.sqrt(6.0 / (n_in + n_out))
        return rng.uniform(-a, a, size=(n_out, n_in)).astype(np.float32)

    for n in linear_names(cfg):
        N, K = _linear_shape(n, cfg)
        sd[f"{n}.weight"] = xavier(N, K)
        bnd = 1.0 / math.sqrt(K)
        sd[f"{n}.bias"] = rng.uniform(-bnd, bnd, size=(N,)).astype(np.float32)
    for n in norm_names(cfg):
        if ln_random:
            sd[f"{n}.a_2"] = rng.uniform(0.5, 1.5, size=(cfg.d_model,)).astype(np.float32)
            sd[f"{n}.b_2"] = rng.uniform(-0.1, 0.1, size=(cfg.d_model,)).astype(np.float32)
        else:
            sd[f"{n}.a_2"] = np.ones(cfg.d_model, np.float32)
            sd[f"{n}.b_2"] = np.zeros(cfg.d_model, np.float32)
    sd["src_embed.0.lut.weight"] = xavier(cfg.src_vocab, cfg.d_model)
    sd["tgt_embed.0.lut.weight"] = xavier(cfg.tgt_vocab, cfg.d_model)
    sd["generator.proj.weight"] = xavier(cfg.tgt_vocab, cfg.d_model)
    bnd = 1.0 / math.sqrt(cfg.d_model)
    sd["generator.proj.bias"] = rng.uniform(-bnd, bnd, size=(cfg.tgt_vocab,)).astype(np.float32)
    if with_pe:
        pe = positional_table(cfg.d_model, cfg.max_len)
        sd["src_embed.1.pe"] = pe[None]
        sd["tgt_embed.1.pe"] = pe[None]
    return sd


def load_checkpoint(path: str, smooth_scales: str | dict | None = None,
                    alpha: float = 0.5) -> dict:
    """Load a reference ``state_dict`` checkpoint without executing pickled code.

    Uses ``torch.load(weights_only=True)``; keys must match :func:`tensor_order`.
    By default smoothing is *not* applied: ``output.py:609-613`` calls ``get_quantized``
    before ``load_state_dict``, which overwrites the smoothed tensors.
    ``smooth_scales`` (a path for :func:`load_act_scales` or its dict) opts in to the
    SmoothQuant fold (:func:`smooth_state_dict`).
    """
    import torch

    raw = torch.load(path, map_location="cpu", weights_only=True)
    sd = {k: v.detach().float().numpy() for k, v in raw.items()}
    missing = [k for k in tensor_order() if k not in sd]
    if missing:
        raise KeyError(f"checkpoint {path} lacks {len(missing)} tensors, e.g. {missing[:3]}")
    if smooth_scales is not None:
        sc = load_act_scales(smooth_scales) if isinstance(smooth_scales, str) else smooth_scales
        sd = smooth_state_dict(sd, sc, alpha)
    return sd


# --------------------------------------------------------------------------------------
# SmoothQuant fold (opt-in)
# --------------------------------------------------------------------------------------

def smooth_groups(cfg: ModelConfig = ModelConfig()) -> list[tuple[str, list[str], str]]:
    """(LayerNorm, linears it feeds, act-scale key) triples that ``smooth_lm``
    (get_quantized_model.py:46-148) smooths, in its module order:

    * encoder layer L: sublayer.0.norm -> self_attn Q/K/V (scales of ``linears.0``),
      sublayer.1.norm -> feed_forward.w_1;
    * decoder layer L: sublayer.0.norm -> self_attn Q/K/V; sublayer.1.norm -> src_attn
      Q/K/V; sublayer.2.norm -> feed_forward.w_1.

    As in the reference, the src_attn K/V weights are scaled too although their input is
    the encoder memory, not that LayerNorm's output (get_quantized_model.py:126-133)."""
    g = []
    for L in range(cfg.n_layers):
        p = f"encoder.layers.{L}"
        g.append((f"{p}.sublayer.0.norm", [f"{p}.self_attn.linears.{i}" for i in range(3)],
                  f"{p}.self_attn.linears.0"))
        g.append((f"{p}.sublayer.1.norm", [f"{p}.feed_forward.w_1"], f"{p}.feed_forward.w_1"))
    for L in range(cfg.n_layers):
        p = f"decoder.layers.{L}"
        g.append((f"{p}.sublayer.0.norm", [f"{p}.self_attn.linears.{i}" for i in range(3)],
                  f"{p}.self_attn.linears.0"))
        g.append((f"{p}.sublayer.1.norm", [f"{p}.src_attn.linears.{i}" for i in range(3)],
                  f"{p}.src_attn.linears.0"))
        g.append((f"{p}.sublayer.2.norm", [f"{p}.feed_forward.w_1"], f"{p}.feed_forward.w_1"))
    return g


def load_act_scales(path: str) -> dict:
    """The per-channel activation maxima SmoothQuant uses (the reference's
    ``scales/transformer_scales.pt``, a dict of fp32 vectors keyed by linear name), loaded
    without executing pickled code (torch.load weights_only=True), or from an .npz."""
    if path.endswith(".npz"):
        with np.load(path) as z:
            return {k: np.asarray(z[k], np.float32) for k in z.files}
    import torch
    raw = torch.load(path, map_location="cpu", weights_only=True)
    return {k: v.detach().float().numpy() for k, v in raw.items()}


def smooth_state_dict(sd: dict, act_scales: dict, alpha: float = 0.5,
                      cfg: ModelConfig = ModelConfig()) -> dict:
    """SmoothQuant folded into the weights at load (smooth_ln_fcs, get_quantized_model.py:
    9-36, applied as smooth_lm does, :46-148): per input channel j of each group,
    ``s_j = clamp(act_max_j^alpha / clamp(max_i |W_ij|, 1e-5)^(1-alpha), 1e-5)`` with the
    weight maximum over all of the group's linears; ``a_2 /= s``, ``b_2 /= s``,
    ``W[:, j] *= s_j``.  Same torch fp32 ops as the reference, so the folded tensors are
    bit-identical to a smoothed reference model's.

    Opt-in: the reference's exported path loads its checkpoint *after* smoothing, which
    undoes it (output.py:609-613), so the default load applies nothing.
    Returns a new dict; ``sd`` is not modified."""
    import torch

    out = dict(sd)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32))
    for ln, fcs, key in smooth_groups(cfg):
        ws = [T(out[f"{n}.weight"]) for n in fcs]
        wmax = torch.cat([w.abs().max(dim=0, keepdim=True)[0] for w in ws], dim=0)
        wmax = wmax.max(dim=0)[0].clamp(min=1e-5)
        s = (T(act_scales[key]).pow(alpha) / wmax.pow(1 - alpha)).clamp(min=1e-5)
        out[f"{ln}.a_2"] = T(out[f"{ln}.a_2"]).div(s).numpy()
        out[f"{ln}.b_2"] = T(out[f"{ln}.b_2"]).div(s).numpy()
        for n, w in zip(fcs, ws):
            out[f"{n}.weight"] = w.mul(s.view(1, -1)).numpy()
    return out
