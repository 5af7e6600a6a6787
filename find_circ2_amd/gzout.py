"""spliced_reads.fastq.gz writer: gzip members compressed on worker threads.

The reference writes the file through one GzipFile at level 9 (find_circ.py:445), which
at genome scale costs more than the whole native read loop.  Here the text is cut into
~4 MiB pieces, each compressed as its own gzip member on a thread pool (zlib releases the
GIL) and written in order; concatenated members are one valid gzip stream (RFC 1952 2.2),
so every gzip reader returns the same text.  Level 1: on the FASTQ text this file holds, zlib's
level 2 compresses 6x faster than level 6 for 13 % more bytes (5.2x instead of 6.0x smaller), and
the native loop's libdeflate (csrc/fc2_deflate.h) at level 1 is another 1.55x faster than at level 2
for 1 % more bytes -- at genome scale the compression would otherwise set the read loop's pace on
the box's CPU quota.  Text is encoded as latin-1, the decoding every
reader of this package uses, so input bytes >= 0x80 (qnames, SEQ/QUAL) are written back as the
same single bytes, as the Python-2 reference writes its byte strings.
"""
from __future__ import annotations

import io
import os
import zlib
from collections import deque
from concurrent.futures import ThreadPoolExecutor


def _member(data: bytes, level: int) -> bytes:
    co = zlib.compressobj(level, zlib.DEFLATED, 16 + zlib.MAX_WBITS)   # gzip header + trailer
    return co.compress(data) + co.flush()


class ParallelGzipWriter(io.TextIOBase):
    def __init__(self, path: str, level: int = 1, threads: int = 0, piece: int = 4 << 20, encoding: str = "latin-1"):
        self.path = path
        self.level = level
        self.piece = piece
        self.threads = threads or min(8, os.cpu_count() or 1)
        self._f = open(path, "wb")
        self._level = level
        self._piece = piece
        self._enc = encoding
        self._buf = []
        self._n = 0
        n = self.threads
        self._pool = ThreadPoolExecutor(max_workers=n)
        self._max_pending = 2 * n
        self._pending = deque()

    def writable(self) -> bool:
        return True

    def write(self, s: str) -> int:
        if s:
            self._buf.append(s)
            self._n += len(s)
            if self._n >= self._piece:
                self._submit()
        return len(s)

    def _submit(self):
        data = "".join(self._buf).encode(self._enc)
        self._buf, self._n = [], 0
        for k in range(0, max(1, len(data)), self._piece):      # a large write becomes several members
            self._pending.append(self._pool.submit(_member, data[k:k + self._piece], self._level))
            while len(self._pending) > self._max_pending:
                self._f.write(self._pending.popleft().result())

    def flush(self):
        pass            # pieces are written as they complete; close() writes the rest

    def hand_over(self) -> str:
        """Give the file to another writer (the native read loop, fc2_caller_set_reads_gz) before
        anything was written: this object then writes nothing, and close() only releases it."""
        if self._buf or self._pending:
            raise ValueError("hand_over after text was written")
        self._f.close()
        self._f = None
        self._pool.shutdown()
        return self.path

    def close(self):
        if self._f is None:
            return
        if self._n or not self._pending:
            self._submit()              # (an empty file still gets one empty member)
        while self._pending:
            self._f.write(self._pending.popleft().result())
        self._pool.shutdown()
        self._f.close()
        self._f = None
        super().close()
