"""Python handle of the native SAM/BAM ingest (include/fc2_ingest.h)."""
from __future__ import annotations

import ctypes
from typing import Dict, List, Tuple

from . import _native as N
from .samio import AlignedSegment, parse_sam_line


class NativeIngest:
    """Streams fragments that carry anchor pairs; counts the rest natively."""

    def __init__(self, path: str, is_bam: bool):
        self.h = ctypes.c_void_p()
        from .native_caller import _check          # the reference's exception types (ValueError, IOError)
        _check(N.lib().fc2_ingest_open(path.encode(), int(is_bam), ctypes.byref(self.h)))
        L = N.lib()
        self.references = [L.fc2_ingest_ref_name(self.h, i).decode("latin-1")
                           for i in range(L.fc2_ingest_n_refs(self.h))]
        self.tid_of: Dict[str, int] = {n: i for i, n in enumerate(self.references)}
        self.counts = N.IngestCounts()
        self.eof = False

    def format(self) -> Tuple[str, str]:
        """(``"sam"`` | ``"bam"``, ``"plain"`` | ``"bgzf"`` | ``"gzip"``), detected from the bytes."""
        comp = ctypes.c_int()
        fmt = N.lib().fc2_ingest_format(self.h, ctypes.byref(comp))
        return ("sam", "bam")[fmt], ("plain", "bgzf", "gzip")[comp.value]

    def getrname(self, tid: int) -> str:
        return self.references[tid]

    def next_chunk(self, asize: int, nolinear: bool, noop: bool, max_frags: int) -> List[List[AlignedSegment]]:
        """Records of the next handed-back fragments (up to max_frags fragments read)."""
        p = N.IngestParams(int(asize), int(bool(nolinear)), int(bool(noop)))
        text = ctypes.c_void_p()
        ln, nh = ctypes.c_uint64(), ctypes.c_uint64()
        eof = ctypes.c_int()
        N.check(N.lib().fc2_ingest_next(self.h, ctypes.byref(p), max_frags, ctypes.byref(self.counts),
                                        ctypes.byref(text), ctypes.byref(ln), ctypes.byref(nh), ctypes.byref(eof)))
        self.eof = bool(eof.value)
        if not ln.value:
            return []
        raw = ctypes.string_at(text, ln.value).decode("latin-1")
        frags = []
        for block in raw.split("\n\n"):
            if block:
                frags.append([parse_sam_line(l, self.tid_of) for l in block.split("\n") if l])
        return frags

    def set_bam_out(self, path: str):
        """-B/--bam: anchor alignments to ``path`` (include/fc2_ingest.h)."""
        N.check(N.lib().fc2_ingest_set_bam_out(self.h, path.encode()))

    def set_gpu_inflate(self, device: int, wait: bool = True):
        """A BGZF input's blocks inflated on GPU ``device`` from the next batch on (include/fc2_ingest.h);
        wait: the device's buffers made now (else meanwhile, the CPU inflating until they are)."""
        N.check(N.lib().fc2_ingest_set_gpu_inflate(self.h, int(device), int(bool(wait))))

    def set_gpu_inflate_from(self, device: int, after_bytes: int):
        """As set_gpu_inflate, with nothing made on the device until ``after_bytes`` of the input were
        read (fc2_ingest_set_gpu_inflate_from; the CLI's default)."""
        N.check(N.lib().fc2_ingest_set_gpu_inflate_from(self.h, int(device), int(after_bytes)))

    def inflate_counts(self) -> Tuple[int, int]:
        """(blocks inflated on the GPU, on the CPU) since set_gpu_inflate."""
        g, c = ctypes.c_uint64(), ctypes.c_uint64()
        N.check(N.lib().fc2_ingest_inflate_counts(self.h, ctypes.byref(g), ctypes.byref(c)))
        return int(g.value), int(c.value)

    def close_bam_out(self):
        N.check(N.lib().fc2_ingest_close_bam_out(self.h))

    def close(self):
        if self.h:
            N.lib().fc2_ingest_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sam_to_bam(sam_path: str, bam_path: str) -> None:
    """BGZF BAM of a SAM file, records encoded as htslib's sam_parse1 does (include/fc2_ingest.h)."""
    N.check(N.lib().fc2_sam_to_bam(sam_path.encode(), bam_path.encode()))
