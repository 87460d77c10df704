"""Greedy decoding and the sentence-sharded multi-GPU driver.

``greedy_decode(model, src, src_mask, max_len, start_symbol)`` has the signature and
result of the reference's decode loops (reference/onnx_reference_inference.py:622-646;
batched form batch_output.py:659-673): ``ys`` starts with ``start_symbol`` and grows by
``max_len - 1`` argmax tokens, with no EOS exit.  The whole loop (encoder, cross K/V,
71 KV-cached decoder steps, generator + argmax) runs on the GPU in one library call.
"""
from __future__ import annotations

import numpy as np

from .model import QtxModel, to_u8_mask
from .weights import PAD


def greedy_decode(model: QtxModel, src, src_mask, max_len: int, start_symbol: int = 0):
    """src int64 [B,S] (numpy or torch), src_mask [B,1,S] bool -> ys int64 [B,max_len]."""
    import torch
    was_numpy = isinstance(src, np.ndarray)
    src_t = torch.from_numpy(np.ascontiguousarray(src)) if was_numpy else src
    B, S = src_t.shape
    srcd = src_t.to(model.device, torch.int64).contiguous()
    md = to_u8_mask(src_mask, model.device).reshape(B, S)
    ys = model.greedy(srcd, md, max_len=max_len, start=start_symbol)
    if was_numpy:
        return ys.cpu().numpy()
    return ys.to(src_t.device)


def make_src_mask(src, pad: int = PAD):
    """Batch.src_mask = (src != pad).unsqueeze(-2)   (batch.py:7)."""
    return (np.asarray(src) != pad)[:, None, :]


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced sentence shard of rank (no data-path collective)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)
