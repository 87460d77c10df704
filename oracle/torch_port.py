"""CPU BASELINE PORT — test / measurement infrastructure only.

Only ``bench.py``'s ``cpu_baseline`` leg (and tests of this file) may import it; the
product path never does.

What it is: the reference's own CPU arithmetic — fp32 fake-quant W8A8 in PyTorch — restated
with torch ops on the host cores, as the reference's modules run it:

* activations per token ``s = max(|x|, 1e-5)/127; q = round(x/s)·s``
  (quant_linear.py:30-43), weights per channel once at load (quant_linear.py:5-17 —
  re-quantizing every forward, as the reference does, is idempotent);
* ``W8A8Linear``: ``F.linear(q_x, q_w, b)``, Q/K/V outputs quantized per token
  (quant_linear.py:111-119, get_quantized_model.py:160-168);
* attention ``softmax(QKᵀ/8, masked -1e9)``, ``P = round(P·127)/127``, ``P·V``
  (attention.py:23-36); LayerNorm with the unbiased std (layer_norm.py:12-15);
* embeddings ``lut·√512 + pe`` and the fp32 generator + first argmax
  (embeddings.py:12-13, generator.py:14-15, onnx_reference_inference.py:640-641).

It follows torch's float evaluation order (MKL/oneDNN GEMMs, torch softmax), not the
canonical order of oracle/qtx_oracle.py, so its tokens can differ from the GPU's at
near-ties; it is a speed baseline, not the parity oracle.  The greedy decode keeps a
K/V cache (the reference recomputes the whole prefix every step,
onnx_reference_inference.py:630-639 — caching makes this baseline faster than the
reference's own loop, i.e. a stricter comparison).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def _qact(x):
    s = x.abs().amax(dim=-1, keepdim=True).clamp(min=1e-5) / 127.0
    return torch.round(x / s) * s


def _qw(w, n_bits=8):
    qmax = 2 ** (n_bits - 1) - 1
    s = w.abs().amax(dim=-1, keepdim=True).clamp(min=1e-5) / qmax
    return torch.round(w / s) * s


class TorchPortModel:
    def __init__(self, sd: dict, n_layers=6, n_heads=8, n_bits=8):
        T = lambda k: torch.from_numpy(np.ascontiguousarray(sd[k], np.float32))
        self.H = n_heads
        self.L = n_layers

        def lin(p):
            return (_qw(T(p + ".weight"), n_bits), T(p + ".bias"))

        def ln(p):
            return (T(p + ".a_2"), T(p + ".b_2"))
        self.enc = []
        for l in range(n_layers):
            p = f"encoder.layers.{l}"
            self.enc.append(dict(att=[lin(f"{p}.self_attn.linears.{i}") for i in range(4)],
                                 w1=lin(f"{p}.feed_forward.w_1"), w2=lin(f"{p}.feed_forward.w_2"),
                                 ln=[ln(f"{p}.sublayer.{i}.norm") for i in range(2)]))
        self.dec = []
        for l in range(n_layers):
            p = f"decoder.layers.{l}"
            self.dec.append(dict(att=[lin(f"{p}.self_attn.linears.{i}") for i in range(4)],
                                 src=[lin(f"{p}.src_attn.linears.{i}") for i in range(4)],
                                 w1=lin(f"{p}.feed_forward.w_1"), w2=lin(f"{p}.feed_forward.w_2"),
                                 ln=[ln(f"{p}.sublayer.{i}.norm") for i in range(3)]))
        self.enc_norm = ln("encoder.norm")
        self.dec_norm = ln("decoder.norm")
        self.src_lut = T("src_embed.0.lut.weight")
        self.tgt_lut = T("tgt_embed.0.lut.weight")
        self.gen = (T("generator.proj.weight"), T("generator.proj.bias"))
        pe = sd.get("src_embed.1.pe")
        if pe is None:
            from qtx.weights import positional_table
            pe = positional_table()
        self.pe = torch.from_numpy(np.ascontiguousarray(np.asarray(pe, np.float32).reshape(-1, 512)))

    # ---- modules -------------------------------------------------------------------
    @staticmethod
    def _linear(p, x, out_quant=False):
        y = F.linear(_qact(x), p[0], p[1])
        return _qact(y) if out_quant else y

    @staticmethod
    def _ln(p, x):
        mean = x.mean(-1, keepdim=True)
        std = x.std(-1, keepdim=True)
        return p[0] * (x - mean) / (std + 1e-6) + p[1]

    def _split(self, x):
        B, T, D = x.shape
        return x.view(B, T, self.H, D // self.H).transpose(1, 2)

    def _attend(self, q, k, v, mask):
        s = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(q.shape[-1])
        s = s.masked_fill(mask == 0, -1e9)
        p = torch.round(s.softmax(dim=-1) * 127.0) / 127.0
        ctx = torch.matmul(p, v)
        B, H, T, dk = ctx.shape
        return ctx.transpose(1, 2).reshape(B, T, H * dk)

    def _ffn(self, L, x, ln):
        h = torch.relu(self._linear(L["w1"], self._ln(ln, x)))
        return x + self._linear(L["w2"], h)

    def embed(self, ids, lut, pos0=0):
        T = ids.shape[1]
        return lut[ids] * math.sqrt(512) + self.pe[pos0:pos0 + T]

    @torch.inference_mode()
    def encode(self, x, src_mask):
        """x [B,S,512], src_mask bool [B,1,S] -> memory [B,S,512]."""
        m = src_mask[:, None]                       # [B,1,1,S]
        for L in self.enc:
            h = self._ln(L["ln"][0], x)
            q, k, v = (self._split(self._linear(L["att"][i], h, True)) for i in range(3))
            x = x + self._linear(L["att"][3], self._attend(q, k, v, m))
            x = self._ffn(L, x, L["ln"][1])
        return self._ln(self.enc_norm, x)

    @torch.inference_mode()
    def greedy_decode(self, src, src_mask, max_len=72, start=0):
        """KV-cached greedy decode: src int64 [B,S], src_mask bool [B,1,S] -> ids [B,max_len]."""
        B = src.shape[0]
        memory = self.encode(self.embed(src, self.src_lut), src_mask)
        sm = src_mask[:, None]
        ck = [(self._split(self._linear(L["src"][1], memory, True)),
               self._split(self._linear(L["src"][2], memory, True))) for L in self.dec]
        cache = [[None, None] for _ in self.dec]
        ys = torch.full((B, 1), start, dtype=torch.int64)
        for t in range(max_len - 1):
            x = self.embed(ys[:, -1:], self.tgt_lut, t)
            one = torch.ones((1, 1, 1, t + 1), dtype=torch.bool)
            for l, L in enumerate(self.dec):
                h = self._ln(L["ln"][0], x)
                q, k, v = (self._split(self._linear(L["att"][i], h, True)) for i in range(3))
                kc, vc = cache[l]
                kc = k if kc is None else torch.cat([kc, k], 2)
                vc = v if vc is None else torch.cat([vc, v], 2)
                cache[l] = [kc, vc]
                x = x + self._linear(L["att"][3], self._attend(q, kc, vc, one))
                h = self._ln(L["ln"][1], x)
                q = self._split(self._linear(L["src"][0], h, True))
                x = x + self._linear(L["src"][3], self._attend(q, ck[l][0], ck[l][1], sm))
                x = self._ffn(L, x, L["ln"][2])
            x = self._ln(self.dec_norm, x[:, -1])
            logp = F.log_softmax(F.linear(x, *self.gen), dim=-1)
            ys = torch.cat([ys, logp.argmax(dim=1, keepdim=True)], 1)
        return ys
