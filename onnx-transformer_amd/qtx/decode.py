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


def greedy_decode_fault(model: QtxModel, src, src_mask, max_len: int, start_symbol: int = 0,
                        fault=None, target_inference_number: int = 1):
    """Greedy decode with one injected fault, the reference campaign's loop
    (parallelized_inject_onnx_transformer.py:536-720): an encoder fault corrupts the single
    encoder run (memory); a decoder fault corrupts only the decoder run of step
    ``target_inference_number - 1`` — every step recomputes the whole prefix, as the
    reference does, so the faulty step changes that step's token and nothing else directly.
    src / src_mask as greedy_decode; returns ys int64 [B, max_len] (numpy)."""
    import torch
    src = np.ascontiguousarray(np.asarray(src), np.int64)
    B, S = src.shape
    dev = model.device
    srcd = torch.from_numpy(src).to(dev)
    md = to_u8_mask(src_mask, dev).reshape(B, S)
    enc_fault = fault if fault is not None and fault.module == 0 else None
    dec_fault = fault if fault is not None and fault.module == 1 else None
    if dec_fault is None:                       # KV-cached fused decode, faulty encoder
        return model.greedy(srcd, md, max_len=max_len, start=start_symbol,
                            fault=enc_fault).cpu().numpy()
    memory = model.encode(model.embed(srcd, "src"), md)
    ys = torch.full((B, 1), int(start_symbol), dtype=torch.int64, device=dev)
    for i in range(max_len - 1):
        T = ys.shape[1]
        tm = torch.tril(torch.ones((T, T), dtype=torch.uint8, device=dev))
        out = model.decode(model.embed(ys, "tgt"), memory, md, tm,
                           fault=dec_fault if i == target_inference_number - 1 else None)
        _, nxt = model.generator(out[:, -1].contiguous(), want_logp=False)
        ys = torch.cat([ys, nxt[:, None]], dim=1)
    return ys.cpu().numpy()


def make_src_mask(src, pad: int = PAD):
    """Batch.src_mask = (src != pad).unsqueeze(-2)   (batch.py:7)."""
    return (np.asarray(src) != pad)[:, None, :]


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced sentence shard of rank (no data-path collective)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)
