"""Multi-GPU sharding of the breakpoint search: one process per GPU, no collective on the data path.

Pairs are independent (``find_breakpoints`` reads only its own span plus the
read-only genome/options, find_circ.py:854-974), so a pair stream is cut into
contiguous batches dealt round-robin to the ranks; every rank scans its batches
on its own GPU with its own genome copy.  The caller needs the per-pair results
back in input order: junction names are given by first appearance
(``SpliceSiteStorage.add``, find_circ.py:681-690) and float weights accumulate
in order (find_circ.py:544, 563, 579).  ``gather_ordered`` moves the 8-byte
result records of every batch to rank 0 over the host process group (gloo) and
restores the input order.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Sequence, Tuple

import numpy as np


def batch_bounds(n: int, batch: int) -> List[Tuple[int, int]]:
    """Contiguous [start, end) batches covering n pairs."""
    if batch <= 0:
        raise ValueError("batch must be positive")
    return [(s, min(n, s + batch)) for s in range(0, n, batch)]


def my_batches(n: int, batch: int, rank: int, world: int) -> List[Tuple[int, int, int]]:
    """(batch_index, start, end) of the batches rank ``rank`` scans (round-robin)."""
    return [(k, s, e) for k, (s, e) in enumerate(batch_bounds(n, batch)) if k % world == rank]


def ordered_merge(parts: Iterable[Sequence[Tuple[int, np.ndarray]]], n_batches: int) -> np.ndarray:
    """Concatenate per-batch result arrays from all ranks in batch (= input) order."""
    by_k: Dict[int, np.ndarray] = {}
    for rank_parts in parts:
        for k, arr in rank_parts:
            if k in by_k:
                raise ValueError("batch %d reported twice" % k)
            by_k[k] = arr
    missing = [k for k in range(n_batches) if k not in by_k]
    if missing:
        raise ValueError("batches missing from the merge: %s" % missing[:8])
    if not by_k:
        return np.zeros(0, np.uint8)
    return np.concatenate([by_k[k] for k in range(n_batches)])


def gather_ordered(local: Sequence[Tuple[int, np.ndarray]], n_batches: int, group=None):
    """Gather every rank's (batch_index, results) to rank 0 and merge in input order.

    Host-side collective over a CPU (gloo) group; returns the merged array on rank
    0 and None elsewhere.  Single-process runs merge locally.
    """
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return ordered_merge([local], n_batches)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    payload = [(int(k), np.ascontiguousarray(a)) for k, a in local]
    out = [None] * world if rank == 0 else None
    dist.gather_object(payload, out, dst=0, group=group)
    if rank != 0:
        return None
    return ordered_merge(out, n_batches)


def round_robin_batch(n: int, world: int, per_rank: int = 4, align: int = 512) -> int:
    """Batch size for dealing n pairs round-robin: about `per_rank` batches per rank (balanced to
    one batch), rounded up to `align` pairs so every batch starts on a 512-pair scan block."""
    if n <= 0:
        return align
    b = -(-n // (max(1, world) * max(1, per_rank)))
    return -(-b // align) * align


def round_bounds(n: int, world: int, per_rank: int = 4, align: int = 512, tail: int = 0) -> List[Tuple[int, int]]:
    """Contiguous [start, end) batches covering n pairs, dealt in rounds of `world` equal batches
    (batch k goes to rank k % world, as in my_batches): `per_rank` rounds of round_robin_batch's
    size, except that with tail = t > 0 the last round is cut into t + 1 rounds of 1/2, 1/4, ...,
    1/2^t, 1/2^t of a batch (each rounded up to `align`).  A rank then copies its results off the
    device in pieces that shrink toward the end of its share: every piece's copy overlaps the scan
    of the next one, and the copy nobody waits behind is 1/2^t of a batch instead of a whole one.
    Results never depend on the cut (pairs are independent, find_circ.py:854-974)."""
    b = round_robin_batch(n, world, per_rank=per_rank, align=align)
    sizes = [b] * max(0, per_rank - 1)
    if tail > 0:
        sizes += [max(align, -(-(b >> j) // align) * align) for j in range(1, tail + 1)]
        sizes.append(sizes[-1])
    else:
        sizes.append(b)
    out, s, i = [], 0, 0
    while s < n:
        size = sizes[min(i, len(sizes) - 1)]
        for _ in range(max(1, world)):
            if s >= n:
                break
            out.append((s, min(n, s + size)))
            s += size
        i += 1
    return out


def my_bounds(bounds: Sequence[Tuple[int, int]], rank: int, world: int) -> List[Tuple[int, int, int]]:
    """(batch_index, start, end) of the batches of `bounds` rank ``rank`` scans (round-robin)."""
    return [(k, s, e) for k, (s, e) in enumerate(bounds) if k % world == rank]


SHM_DIR = "/dev/shm"
SHM_HEADROOM = 64 << 20


def _free_bytes(path: str) -> int:
    try:
        st = os.statvfs(path)
        return st.f_bavail * st.f_frsize
    except OSError:
        return 0


class _FileSegment:
    """A MAP_SHARED mapping of a file outside /dev/shm, for a node whose /dev/shm cannot hold the
    merge buffer (a container's 64 MB default against the ~0.7 GB of configs[3]'s three forms):
    every rank on the node maps the same file, which page-locks like the tmpfs segment.  Named
    ``file:<path>`` so the attaching ranks know the kind."""
    PREFIX = "file:"

    def __init__(self, name: str = None, create: bool = False, size: int = 0):
        import mmap
        import tempfile
        if create:
            d = tempfile.gettempdir()
            if _free_bytes(d) < size + SHM_HEADROOM:
                raise OSError("no room for a %d-byte merge buffer in %s or %s" % (size, SHM_DIR, d))
            fd, path = tempfile.mkstemp(prefix="fc2_merge_", dir=d)
            os.ftruncate(fd, size)
        else:
            path = name[len(self.PREFIX):]
            fd = os.open(path, os.O_RDWR)
            size = os.fstat(fd).st_size
        try:
            self._mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.buf = memoryview(self._mm)
        self.name = self.PREFIX + path
        self._path = path

    def close(self):
        self.buf.release()
        self._mm.close()

    def unlink(self):
        os.unlink(self._path)


def _segment(name: str = None, create: bool = False, size: int = 0):
    """The node-local segment behind a merge buffer: POSIX shared memory (/dev/shm) when it has room,
    else a shared file mapping (_FileSegment); attaching ranks follow the creator's choice by name."""
    if (create and _free_bytes(SHM_DIR) < size + SHM_HEADROOM) or \
            (not create and name.startswith(_FileSegment.PREFIX)):
        return _FileSegment(name, create, size)
    from multiprocessing import resource_tracker, shared_memory
    shm = shared_memory.SharedMemory(name=name, create=create, size=size)
    if not create:
        # the attaching process must not unlink the segment when it exits (Python < 3.13 tracks
        # every attach as if it owned the segment)
        try:
            resource_tracker.unregister(shm._name, "shared_memory")
        except Exception:
            pass
    return shm


class SharedResults:
    """Node-local ordered merge of per-pair results: ONE host buffer of n 8-byte ``fc2_result``
    records in /dev/shm (or a shared file mapping when /dev/shm is too small, _segment) that every
    rank on the node maps.  A rank copies each of its batches'
    results (D2H, on its own stream) straight to the batch's input offset, so after a barrier rank
    0 holds every result in input order without gathering or reordering anything -- the order
    ``SpliceSiteStorage`` naming (find_circ.py:681-690) and the float weight sums (:544, :563,
    :579) need.  The buffer is page-locked with ``fc2_host_register`` when a GPU is present, so the
    copies run asynchronously at PCIe rate.

    Create on rank 0 (``create=True``), then the others attach by ``name`` (broadcast it);
    ``close()`` on every rank, rank 0 last (it unlinks)."""

    def __init__(self, n: int, name: str = None, create: bool = False, pin: bool = False):
        self.n = int(n)
        self.creator = create
        self.shm = _segment(name, create, max(8, 8 * self.n))
        self.name = self.shm.name
        self.array = np.ndarray((self.n,), np.int64, buffer=self.shm.buf)
        self._pinned = False
        if pin and self.n:
            from . import _native as N
            N.check(N.lib().fc2_host_register(self.array.ctypes.data, 8 * self.n))
            self._pinned = True
        import torch
        self.tensor = torch.from_numpy(self.array)

    def close(self):
        if self.shm is None:
            return
        if self._pinned:
            from . import _native as N
            N.lib().fc2_host_unregister(self.array.ctypes.data)
            self._pinned = False
        self.tensor = None
        self.array = None
        self.shm.close()
        if self.creator:
            self.shm.unlink()
        self.shm = None


class SharedCompactResults(SharedResults):
    """The same node-local ordered merge in a compact transfer form of the results (include/fc2_bp.h
    "compact results", canonical mode, `width` 4 or 2 bytes per pair): one /dev/shm segment holding
    ``words`` [n] (at each batch's input offset), per batch ``cap`` escape slots (``N.ESCAPE_DTYPE``,
    indices relative to the batch start) and the batch's escape count.  A half or a quarter of the
    bytes of the 8-byte merge cross PCIe and land in host memory; ``merged()`` expands the whole
    stream (fc2_result_expand) where a consumer wants 8-byte words, and fc2_caller_submit_compact
    takes the form as it is."""

    def __init__(self, n: int, bounds: Sequence[Tuple[int, int]], cap: int, name: str = None, create: bool = False,
                 pin: bool = False, width: int = 4):
        from . import _native as N
        if width not in (2, 4):
            raise ValueError("width is 2 or 4")
        self.n, self.bounds, self.cap, self.width = int(n), list(bounds), int(cap), width
        nb = len(self.bounds)
        self._w_bytes = (width * self.n + 63) // 64 * 64
        self._e_bytes = 16 * (self.cap + 1) * nb    # per batch: cap escape slots, then the count's slot
        size = max(64, self._w_bytes + self._e_bytes)
        self.creator = create
        self.shm = _segment(name, create, size)
        self.name = self.shm.name
        buf = self.shm.buf
        self.words = np.ndarray((self.n,), np.uint16 if width == 2 else np.uint32, buffer=buf)
        # batch k's block mirrors the device CompactResults.esc_block: escape slots, then the count in
        # the low 4 bytes of one more slot; one D2H copy per batch carries both
        self.esc_blocks = np.ndarray((nb, self.cap + 1), N.ESCAPE_DTYPE, buffer=buf, offset=self._w_bytes)
        self.esc = self.esc_blocks[:, :self.cap]
        self.esc_count = np.ndarray((nb,), np.int32, buffer=buf, offset=self._w_bytes + 16 * self.cap,
                                    strides=(16 * (self.cap + 1),)) if nb else np.zeros(0, np.int32)
        self.array = np.ndarray((size,), np.uint8, buffer=buf)      # the whole segment (pinning, poisoning)
        self._pinned = False
        if pin and size:
            N.check(N.lib().fc2_host_register(self.array.ctypes.data, size))
            self._pinned = True
        import torch
        self.tensor = torch.from_numpy(self.array)
        self.words_t = torch.from_numpy(self.words.view(np.int16 if width == 2 else np.int32))
        self.esc_t = torch.from_numpy(self.esc_blocks.view(np.uint8).reshape(nb, 16 * (self.cap + 1)))

    def escapes(self) -> np.ndarray:
        """Every batch's escapes with stream indices; ValueError if a batch overflowed its slots."""
        parts = []
        for k, (lo, _) in enumerate(self.bounds):
            c = int(self.esc_count[k])
            if c < 0:
                raise ValueError("batch %d: its escape count was never written" % k)
            if c > self.cap:
                raise ValueError("batch %d has %d escapes, %d slots" % (k, c, self.cap))
            e = self.esc[k, :c].copy()
            e["index"] += lo
            parts.append(e)
        from . import _native as N
        return np.concatenate(parts) if parts else np.zeros(0, N.ESCAPE_DTYPE)

    def merged(self, options, n_threads: int = 0) -> np.ndarray:
        from .hotpath import expand
        return expand(options, self.words, self.escapes(), n_threads=n_threads)

    def close(self):
        self.words = self.esc = self.esc_blocks = self.esc_count = None
        self.words_t = self.esc_t = None
        super().close()


def broadcast_name(name, group=None) -> str:
    """Rank 0's shared-memory segment name on every rank (host group)."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return name
    obj = [name]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def gather_ints(x: int, group=None) -> List[int]:
    """Every rank's Python int, in rank order, on every rank (host group); [x] without one."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [int(x)]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, int(x), group=group)
    return [int(v) for v in out]


def max_over_ranks(x: float, device=None, group=None) -> float:
    """Max of a scalar over ranks (timing); works on the nccl (GPU tensor) and gloo (CPU tensor) backends."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x
    dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
