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
    model.check()
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
        ys = model.greedy(srcd, md, max_len=max_len, start=start_symbol, fault=enc_fault)
        model.check()
        return ys.cpu().numpy()
    memory = model.encode(model.embed(srcd, "src"), md)
    model.check()                               # the encode's device errors, before the loop
    ys = torch.full((B, 1), int(start_symbol), dtype=torch.int64, device=dev)
    for i in range(max_len - 1):
        T = ys.shape[1]
        tm = torch.tril(torch.ones((T, T), dtype=torch.uint8, device=dev))
        out = model.decode(model.embed(ys, "tgt"), memory, md, tm,
                           fault=dec_fault if i == target_inference_number - 1 else None)
        _, nxt = model.generator(out[:, -1].contiguous(), want_logp=False)
        ys = torch.cat([ys, nxt[:, None]], dim=1)
    model.check()
    return ys.cpu().numpy()


def make_src_mask(src, pad: int = PAD):
    """Batch.src_mask = (src != pad).unsqueeze(-2)   (batch.py:7)."""
    return (np.asarray(src) != pad)[:, None, :]


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced sentence shard of rank (no data-path collective)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def length_sorted_shards(lengths, world: int):
    """SURVEY §8e's partition: sentences sorted by source length (longest first, stable),
    dealt to ranks as contiguous balanced chunks (:func:`shard_bounds`), so every rank
    gets sentences of similar length.  Returns one index array per rank."""
    order = np.argsort(-np.asarray(lengths), kind="stable")
    return [order[slice(*shard_bounds(len(order), world, r))] for r in range(world)]


def gather_ids(dist, ids_local, idx_local, n_global: int, world: int):
    """All-gather every rank's decoded ids (int64 [n_r, L], rows ``idx_local`` of the
    global batch) back into global order on every rank: one padded all_gather of the ids
    and one of the indices (≈0.6 MB for 2048 × 72 ids) after the timed region — not on the
    data path.  Works on gloo (CPU tensors) and nccl/RCCL (device tensors)."""
    import torch
    dev = ids_local.device
    L = ids_local.shape[1]
    n = torch.tensor([ids_local.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    mx = int(max(int(s.item()) for s in sizes))
    buf = torch.full((mx, L), -1, dtype=torch.int64, device=dev)
    buf[:ids_local.shape[0]] = ids_local
    ib = torch.full((mx,), -1, dtype=torch.int64, device=dev)
    ib[:ids_local.shape[0]] = torch.as_tensor(np.asarray(idx_local), dtype=torch.int64, device=dev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    iparts = [torch.empty_like(ib) for _ in range(world)]
    dist.all_gather(parts, buf)
    dist.all_gather(iparts, ib)
    out = np.full((n_global, L), -1, np.int64)
    for p, ip, s in zip(parts, iparts, sizes):
        k = int(s.item())
        out[ip[:k].cpu().numpy()] = p[:k].cpu().numpy()
    return out
