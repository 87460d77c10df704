"""Sentence sharding across ranks: CPU, gloo, world_size 2.

The multi-GPU path partitions the sentence batch with ``qtx.decode.shard_bounds`` and has
no data-path collective; each rank decodes its shard independently.  Here two gloo ranks
decode their shards with the CPU oracle (the checker — same arithmetic as the HIP path)
and gather the token ids; the result must equal the single-process full-batch decode
(per-token quantization ⇒ batch-composition invariance), and the max-over-ranks timing
reduction bench.py uses must work on the gloo backend.
"""
import os
import socket

import numpy as np
import pytest

from qtx.decode import length_sorted_shards, make_src_mask, shard_bounds


def test_length_sorted_shards():
    lens = np.array([5, 9, 9, 2, 7, 12, 3])
    sh = length_sorted_shards(lens, 3)
    assert sorted(np.concatenate(sh).tolist()) == list(range(7))
    assert [len(s) for s in sh] == [3, 2, 2]
    assert sh[0].tolist() == [5, 1, 2] and sh[1].tolist() == [4, 0]   # longest first, stable


def test_shard_bounds_partition():
    for n in (0, 1, 7, 32, 2048, 2049):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(B=5, S=12, seed=3):
    rng = np.random.default_rng(seed)
    src = np.full((B, S), 2, np.int64)
    for b, n in enumerate(rng.integers(4, S + 1, B)):
        src[b, 0] = 0
        src[b, 1:n - 1] = rng.integers(4, 5337, n - 2)
        src[b, n - 1] = 1
    return src


def _rank(rank, world, port, out_dir):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (repo, os.path.join(repo, "onnx-transformer_amd")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from oracle.qtx_oracle import OracleModel
    from qtx.decode import gather_ids, length_sorted_shards, make_src_mask
    from qtx.weights import ModelConfig, synthetic_state_dict

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    cfg = ModelConfig(n_layers=2)
    om = OracleModel(synthetic_state_dict(20241223, cfg), n_layers=2)
    src = _batch()
    # bench.py's partition and gather: length-sorted shards, padded all_gather
    idx = length_sorted_shards((src != 2).sum(1), world)[rank]
    ys = om.greedy_decode(src[idx], make_src_mask(src[idx]), 6)
    full = gather_ids(dist, torch.from_numpy(ys), idx, len(src), world)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)                 # bench.py's max-over-ranks
    if rank == 0:
        np.save(os.path.join(out_dir, "sharded.npy"), full)
        np.save(os.path.join(out_dir, "tmax.npy"), t.numpy())
    dist.destroy_process_group()


def test_sharded_decode_equals_full_batch(tmp_path):
    import torch.multiprocessing as mp
    from oracle.qtx_oracle import OracleModel
    from qtx.weights import ModelConfig, synthetic_state_dict

    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    sharded = np.load(tmp_path / "sharded.npy")
    assert float(np.load(tmp_path / "tmax.npy")[0]) == world
    om = OracleModel(synthetic_state_dict(20241223, ModelConfig(n_layers=2)), n_layers=2)
    src = _batch()
    full = om.greedy_decode(src, make_src_mask(src), 6)
    np.testing.assert_array_equal(sharded, full)


@pytest.mark.gpu
def test_sharded_gpu_decode_equals_full_batch():
    """On the GPU: each shard decoded separately (as each rank would) equals the batch."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from qtx.decode import greedy_decode
    from qtx.model import QtxModel
    from qtx.weights import ModelConfig, synthetic_state_dict
    m = QtxModel(synthetic_state_dict(20241223, ModelConfig()), ModelConfig())
    src = _batch(B=9, S=20, seed=4)
    mask = make_src_mask(src)
    full = greedy_decode(m, src, mask, 24, 0)
    for world in (2, 4):
        parts = []
        for r in range(world):
            lo, hi = shard_bounds(len(src), world, r)
            parts.append(greedy_decode(m, src[lo:hi], mask[lo:hi], 24, 0))
        np.testing.assert_array_equal(np.concatenate(parts), full)
