"""gloo tests (CPU, world sizes 2, 4 and 8) of the multi-GPU sharding logic (find_circ2_amd/shard.py).

Each rank "scans" its round-robin batches with a deterministic stand-in for the
kernel (per-pair results are a pure function of the pair, as find_breakpoints
is), results are gathered to rank 0 and merged in input order; the merged array
must equal a sequential single-process scan.  The timing max-over-ranks used by
bench.py is checked on gloo too.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from find_circ2_amd import shard


def fake_scan(pairs: np.ndarray) -> np.ndarray:
    # any pure per-pair function stands in for the kernel (8-byte records)
    x = pairs.astype(np.uint64)
    return (x * np.uint64(0x9E3779B97F4A7C15)) ^ (x >> np.uint64(7))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, batch, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pairs = np.arange(n, dtype=np.int64) * 31 + 7
    mine = shard.my_batches(n, batch, rank, world)
    local = [(k, fake_scan(pairs[s:e])) for k, s, e in mine]
    merged = shard.gather_ordered(local, len(shard.batch_bounds(n, batch)))
    t = shard.max_over_ranks(float(rank + 1))
    if rank == 0:
        q.put((merged, t))
    dist.barrier()
    dist.destroy_process_group()


# world 2 over every edge case; 4 and 8 (the node's GPU count) over the cases where some ranks get no
# batch (n < world batches) and where every rank gets several
@pytest.mark.parametrize("world,n,batch", [(2, 1000, 64), (2, 10, 100), (2, 999, 1), (2, 0, 8),
                                           (4, 1000, 64), (4, 10, 4), (8, 1000, 64), (8, 999, 1), (8, 10, 4)])
def test_gloo_ranks_ordered_merge(world, n, batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    merged, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    expect = fake_scan(np.arange(n, dtype=np.int64) * 31 + 7)
    assert np.array_equal(merged, expect)
    assert t == float(world)


def test_batches_cover_and_partition():
    for n, batch, world in [(1000, 64, 8), (7, 3, 2), (0, 5, 4)]:
        seen = []
        for r in range(world):
            seen += [(s, e) for _, s, e in shard.my_batches(n, batch, r, world)]
        seen.sort()
        assert sum(e - s for s, e in seen) == n
        assert all(seen[i][1] == seen[i + 1][0] for i in range(len(seen) - 1))
    with pytest.raises(ValueError):
        shard.ordered_merge([[(0, np.zeros(1))], [(0, np.zeros(1))]], 1)
    with pytest.raises(ValueError):
        shard.ordered_merge([[(0, np.zeros(1))]], 2)


def _shm_worker(rank, world, port, n, batch, q, file_seg=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if file_seg:                                 # a node whose /dev/shm has no room: the file fallback
        shard.SHM_DIR = "/nonexistent"
    pairs = np.arange(n, dtype=np.int64) * 31 + 7
    merged = shard.SharedResults(n, create=True) if rank == 0 else None
    name = shard.broadcast_name(merged.name if rank == 0 else None)
    assert name.startswith("file:") == file_seg
    if rank != 0:
        merged = shard.SharedResults(n, name=name)
    dist.barrier()
    if rank == 0:
        merged.array[:] = -1                     # poison: every slot must be written by some rank
    dist.barrier()
    for _, s, e in shard.my_batches(n, batch, rank, world):
        merged.array[s:e] = fake_scan(pairs[s:e]).view(np.int64)
    dist.barrier()
    if rank == 0:
        q.put(merged.array.copy())
    dist.barrier()
    merged.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("file_seg", [False, True], ids=["shm", "file"])
@pytest.mark.parametrize("world,n", [(2, 1000), (2, 1), (2, 0), (4, 1000), (8, 5000), (8, 1)])
def test_gloo_ranks_shared_memory_merge(world, n, file_seg):
    """bench.py's configs[3] merge (shard.SharedResults): ranks write their round-robin batches'
    results into one node-local buffer at input offsets; rank 0 reads them in input order -- in
    /dev/shm, or in a shared file mapping when /dev/shm has no room (shard._segment)."""
    batch = shard.round_robin_batch(n, world, per_rank=3, align=64)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shm_worker, args=(r, world, port, n, batch, q, file_seg)) for r in range(world)]
    for p in procs:
        p.start()
    merged = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(merged, fake_scan(np.arange(n, dtype=np.int64) * 31 + 7).view(np.int64))


def test_round_robin_batch_balance():
    for n, world in [(50_000_000, 1), (50_000_000, 8), (1_000_000, 2), (513, 4), (1, 8)]:
        b = shard.round_robin_batch(n, world)
        assert b % 512 == 0 and b > 0
        counts = [sum(e - s for _, s, e in shard.my_batches(n, b, r, world)) for r in range(world)]
        assert sum(counts) == n
        assert max(counts) - min(counts) <= b


@pytest.mark.parametrize("tail", [0, 1, 3])
def test_round_bounds_cover_and_shrink(tail):
    for n, world, per_rank in [(50_000_000, 1, 8), (50_000_000, 8, 2), (1_000_000, 2, 4), (513, 4, 2), (1, 8, 2)]:
        bounds = shard.round_bounds(n, world, per_rank=per_rank, tail=tail)
        assert bounds[0][0] == 0 and bounds[-1][1] == n
        assert all(bounds[k][1] == bounds[k + 1][0] for k in range(len(bounds) - 1))
        assert all(e > s and s % 512 == 0 for s, e in bounds)
        b = shard.round_robin_batch(n, world, per_rank=per_rank)
        counts = [sum(e - s for _, s, e in shard.my_bounds(bounds, r, world)) for r in range(world)]
        assert sum(counts) == n and max(counts) - min(counts) <= b
        if tail:
            # the stream ends on a piece of 1/2^tail of a batch
            assert bounds[-1][1] - bounds[-1][0] <= max(512, -(-(b >> tail) // 512) * 512)
        if not tail:
            assert bounds == shard.batch_bounds(n, b)


def _compact_worker(rank, world, port, n, batch, q, width, tail=-1):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_compact_results import pack, sample_words
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    words8 = sample_words(n, 77)                 # the stream's 8-byte results (every rank can derive them)
    # tail >= 0: the strong-scaling stream's rounds (shard.round_bounds, as bench.strong_scaling deals them)
    bounds = shard.batch_bounds(n, batch) if tail < 0 else (shard.round_bounds(n, world, per_rank=3, align=64, tail=tail)
                                                           if n else [])
    cap = max([1, batch] + [e - s for s, e in bounds])
    merged = shard.SharedCompactResults(n, bounds, cap, create=True, width=width) if rank == 0 else None
    name = shard.broadcast_name(merged.name if rank == 0 else None)
    if rank != 0:
        merged = shard.SharedCompactResults(n, bounds, cap, name=name, width=width)
    dist.barrier()
    if rank == 0:
        merged.words[:] = 0x5A5A
        merged.esc_count[:] = -1
    dist.barrier()
    for k, s, e in shard.my_bounds(bounds, rank, world):
        c, esc = pack(words8[s:e], width)       # what fc2_result_compact_launch writes for the batch
        merged.words[s:e] = c
        merged.esc[k, :len(esc)] = esc          # batch-relative indices, as the device writes them
        merged.esc_count[k] = len(esc)
    csum = sum(shard.gather_ints(rank + 10))
    dist.barrier()
    if rank == 0:
        from find_circ2_amd import Options
        q.put((merged.merged(Options()), words8, csum))
    dist.barrier()
    merged.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("width", [4, 2])
@pytest.mark.parametrize("world,n,tail", [(2, 5000, -1), (2, 700, -1), (2, 0, -1), (4, 5000, -1), (8, 5000, -1),
                                          (8, 700, -1), (2, 5000, 3), (4, 5000, 3), (8, 20000, 3), (8, 700, 1)])
def test_gloo_ranks_compact_merge(world, n, tail, width):
    """bench.py's configs[3] merge in a compact transfer form (shard.SharedCompactResults, 4 and 2 bytes):
    words at input offsets, escapes per batch; rank 0's expansion equals the stream's 8-byte results.
    tail >= 0: the strong-scaling layout (shard.round_bounds with shrinking tail rounds)."""
    batch = shard.round_robin_batch(n, world, per_rank=3, align=64)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_compact_worker, args=(r, world, port, n, batch, q, width, tail))
             for r in range(world)]
    for p in procs:
        p.start()
    merged, words8, csum = q.get(timeout=240)
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert np.array_equal(merged, words8)
    assert csum == sum(r + 10 for r in range(world))
