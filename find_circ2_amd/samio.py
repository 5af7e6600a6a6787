"""SAM / BAM input for the caller (pysam is not available in this image).

Provides the subset of ``pysam.AlignedSegment`` / ``pysam.Samfile`` that
find_circ.py reads (find_circ.py:461-477, 809-852, 976-1140, 1442-1486):
``qname, flag, is_* flags, tid, pos, aend, cigar, seq, query, qual, tags,
get_tag, has_tag`` and ``getrname``.  Semantics follow the SAM spec as pysam
exposes it:

* ``pos`` 0-based; ``aend`` = pos + reference span (M/D/N/=/X), None if unmapped
* ``cigar`` = list of (op, length), op codes M0 I1 D2 N3 S4 H5 P6 =7 X8
* ``seq`` = SAM SEQ (None for '*'); ``query`` = SEQ without soft clips
* ``qual`` = SAM QUAL string (None for '*')
"""
from __future__ import annotations

import array
import gzip
import io
import re
import struct
import sys
import zlib
from typing import Dict, Iterator, List, Optional, Tuple

_CIGAR_RE = re.compile(r"(\d+)([MIDNSHP=X])")
_CIGAR_OPS = {"M": 0, "I": 1, "D": 2, "N": 3, "S": 4, "H": 5, "P": 6, "=": 7, "X": 8}
_REF_OPS = (0, 2, 3, 7, 8)


class AlignedSegment:
    __slots__ = ("qname", "flag", "tid", "pos", "mapq", "cigar", "seq", "qual", "tags", "_aend")

    def __init__(self, qname, flag, tid, pos, mapq, cigar, seq, qual, tags):
        self.qname = qname
        self.flag = flag
        self.tid = tid
        self.pos = pos
        self.mapq = mapq
        self.cigar = cigar
        self.seq = seq
        self.qual = qual
        self.tags = tags
        self._aend = -1

    # flags (SAM spec §1.4)
    is_paired = property(lambda self: bool(self.flag & 0x1))
    is_proper_pair = property(lambda self: bool(self.flag & 0x2))
    is_unmapped = property(lambda self: bool(self.flag & 0x4))
    mate_is_unmapped = property(lambda self: bool(self.flag & 0x8))
    is_reverse = property(lambda self: bool(self.flag & 0x10))
    mate_is_reverse = property(lambda self: bool(self.flag & 0x20))
    is_read1 = property(lambda self: bool(self.flag & 0x40))
    is_read2 = property(lambda self: bool(self.flag & 0x80))
    is_secondary = property(lambda self: bool(self.flag & 0x100))
    is_qcfail = property(lambda self: bool(self.flag & 0x200))
    is_duplicate = property(lambda self: bool(self.flag & 0x400))
    is_supplementary = property(lambda self: bool(self.flag & 0x800))

    @property
    def aend(self):
        if self._aend == -1:
            if self.is_unmapped or not self.cigar:
                self._aend = None
            else:
                self._aend = self.pos + sum(n for op, n in self.cigar if op in _REF_OPS)
        return self._aend

    @property
    def query(self):
        """Aligned part of SEQ (soft clips removed), pysam's query_alignment_sequence."""
        if self.seq is None:
            return None
        s = 0
        for op, n in self.cigar:
            if op == 4:
                s += n
            elif op != 5:
                break
        e = len(self.seq)
        for op, n in reversed(self.cigar):
            if op == 4:
                e -= n
            elif op != 5:
                break
        return self.seq[s:e]

    def get_tag(self, tag):
        for t, v in self.tags:
            if t == tag:
                return v
        raise KeyError("tag '%s' not present" % tag)

    def has_tag(self, tag):
        return any(t == tag for t, _ in self.tags)

    def __repr__(self):
        return "AlignedSegment(%s flag=%d tid=%d pos=%d cigar=%s)" % (self.qname, self.flag, self.tid, self.pos,
                                                                      self.cigar)


def parse_cigar(s: str) -> List[Tuple[int, int]]:
    if s == "*":
        return []
    return [(_CIGAR_OPS[op], int(n)) for n, op in _CIGAR_RE.findall(s)]


def parse_sam_line(line: str, tid_of: Dict[str, int]) -> AlignedSegment:
    """One SAM text line -> AlignedSegment (reference names resolved through tid_of)."""
    f = line.rstrip("\r\n").split("\t")
    if len(f) < 11:
        raise ValueError("malformed SAM line: %r" % line[:80])
    rname = f[2]
    tid = -1 if rname == "*" else tid_of.get(rname, -1)
    tags = []
    for t in f[11:]:
        tg, typ, val = t.split(":", 2)
        tags.append((tg, _tag_value(typ, val)))
    return AlignedSegment(f[0], int(f[1]), tid, int(f[3]) - 1, int(f[4]), parse_cigar(f[5]),
                          None if f[9] == "*" else f[9], None if f[10] == "*" else f[10], tags)


def _float32(v: float) -> float:
    """The float32 htslib stores for a 'f' value (pysam hands it back widened to a double)."""
    try:
        return struct.unpack("<f", struct.pack("<f", v))[0]
    except OverflowError:     # C's narrowing of an out-of-range double
        return float("inf") if v > 0 else float("-inf")


_B_CODES = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}


def _tag_value(typ: str, val: str):
    """A SAM text tag value as pysam's get_tag returns it: 'i' an int, 'f' a float (rounded to the
    float32 htslib keeps), 'B' an array.array, anything else (A, Z, H) a str."""
    if typ == "i":
        return int(val)
    if typ == "f":
        return _float32(float(val))
    if typ == "B":
        parts = val.split(",")
        conv = float if parts[0] == "f" else int
        return array.array(_B_CODES.get(parts[0], "i"), [conv(x) for x in parts[1:]])
    return val            # Z, A, H


class _Prefixed(io.RawIOBase):
    """``head`` bytes (already read to detect the format: a pipe cannot be rewound), then ``rest``."""

    def __init__(self, head: bytes, rest):
        self._head = memoryview(head)
        self._rest = rest

    def readable(self):
        return True

    def readinto(self, b):
        if len(self._head):
            n = min(len(b), len(self._head))
            b[:n] = self._head[:n]
            self._head = self._head[n:]
            return n
        data = self._rest.read(len(b))
        b[:len(data)] = data
        return len(data)


class _Inflated(io.RawIOBase):
    """The decompressed bytes of a gzip / BGZF stream, its failures as htslib reports them: a
    member cut short is an IOError ("truncated file"), a corrupt one an IOError too, not zlib's own
    error class."""

    def __init__(self, raw):
        self._gz = gzip.GzipFile(fileobj=raw, mode="rb")

    def readable(self):
        return True

    def readinto(self, b):
        try:
            data = self._gz.read(len(b))
        except EOFError as ex:
            raise IOError("truncated file: %s" % ex)
        except zlib.error as ex:
            raise IOError("corrupt compressed data: %s" % ex)
        b[:len(data)] = data
        return len(data)

    def close(self):
        try:
            self._gz.close()
        finally:
            super().close()


def _read_upto(fh, n: int) -> bytes:
    out = b""
    while len(out) < n:
        d = fh.read(n - len(out))
        if not d:
            break
        out += d
    return out


def sniff(raw) -> Tuple[str, str, object]:
    """Detect the input format from its first bytes, as htslib's hts_detect_format does for the
    reference's pysam.Samfile(path | '-', 'r' | 'rb') (find_circ.py:461-469): gzip (BGZF or not)
    or plain bytes, holding BAM ("BAM\\1") or SAM text.  Returns (format, compression, stream of
    the decompressed bytes from the start)."""
    head = _read_upto(raw, 18)
    stream = io.BufferedReader(_Prefixed(head, raw), 1 << 20)
    comp = "plain"
    if head[:2] == b"\x1f\x8b":
        comp = "bgzf" if (len(head) >= 14 and head[3] & 4 and head[12:14] == b"BC") else "gzip"
        stream = io.BufferedReader(_Inflated(stream), 1 << 20)
    magic = stream.peek(4)[:4]
    if len(magic) < 4 and magic:
        magic = _read_upto(stream, 4)
        stream = io.BufferedReader(_Prefixed(magic, stream), 1 << 20)
    if magic == b"CRAM":
        raise ValueError("CRAM input is not supported (convert it to BAM or SAM)")
    return ("bam" if magic == b"BAM\1" else "sam"), comp, stream


class AlignmentFile:
    """Sequential reader of SAM text or BAM, from a path or '-' (stdin).  ``mode`` is the
    reference's hint ('r' / 'rb', find_circ.py:463-469); as in htslib it does not decide the
    format, the bytes do (``sniff``)."""

    def __init__(self, path: str, mode: str = "r"):
        self.path = path
        self.references: List[str] = []
        self.lengths: List[int] = []
        self.header_lines: List[str] = []
        self._tid: Dict[str, int] = {}
        if path == "-":
            raw = sys.stdin.buffer
        else:
            raw = open(path, "rb")
        self._raw = raw
        fmt, self.compression, stream = sniff(raw)
        self.format = fmt
        self._bam = fmt == "bam"
        if self._bam:
            self._fh = stream
            self._read_bam_header()
        else:
            self._fh = io.TextIOWrapper(stream, encoding="latin-1", newline="\n")
            self._pending = None
            self._read_sam_header()
        if not self.references:       # pysam's check_sq (on by default): no @SQ -> ValueError
            self.close()
            raise ValueError("file has no sequences defined (mode='%s') - is it SAM/BAM format? Consider "
                             "opening with check_sq=False" % mode)

    # ------------------------------------------------------------------ SAM
    def _read_sam_header(self):
        for line in self._fh:
            if not line.startswith("@"):
                self._pending = line
                break
            self.header_lines.append(line.rstrip("\n"))
            if line.startswith("@SQ"):
                d = dict(kv.split(":", 1) for kv in line.rstrip("\r\n").split("\t")[1:] if ":" in kv)
                self._tid[d["SN"]] = len(self.references)
                self.references.append(d["SN"])
                self.lengths.append(int(d.get("LN", 0)))

    def _parse_sam(self, line: str) -> AlignedSegment:
        try:
            return parse_sam_line(line, self._tid)
        except (IndexError, KeyError) as ex:      # htslib: "parse error" / unrecognized reference name
            raise ValueError("SAM parse error: %s in %r" % (ex, line[:80]))

    # ------------------------------------------------------------------ BAM
    def _read(self, n, at_record=False):
        """n bytes of the BAM stream.  EOFError only for a clean end (nothing left where a record
        would start); a stream cut short inside a record or a gzip member is an IOError, as
        htslib reports a truncated file."""
        if n < 0:
            raise ValueError("invalid BAM length field %d" % n)
        try:
            if n <= 1 << 24:
                b = self._fh.read(n)
            else:                       # a corrupt length: no up-front allocation of its size
                parts, got = [], 0
                while got < n:
                    part = self._fh.read(min(1 << 24, n - got))
                    if not part:
                        break
                    parts.append(part)
                    got += len(part)
                b = b"".join(parts)
        except EOFError as ex:          # gzip: "Compressed file ended before the end-of-stream marker ..."
            raise IOError("truncated file: %s" % ex)
        if len(b) != n:
            if at_record and not b:
                raise EOFError
            raise IOError("truncated file")
        return b

    def _read_bam_header(self):
        if self._read(4) != b"BAM\1":
            raise ValueError("not a BAM file")
        l_text, = struct.unpack("<i", self._read(4))
        text = self._read(l_text).decode("latin-1")
        self.header_lines = [l for l in text.split("\n") if l]
        n_ref, = struct.unpack("<i", self._read(4))
        for _ in range(n_ref):
            l_name, = struct.unpack("<i", self._read(4))
            name = self._read(l_name)[:-1].decode("latin-1")
            l_ref, = struct.unpack("<i", self._read(4))
            self._tid[name] = len(self.references)
            self.references.append(name)
            self.lengths.append(l_ref)

    _SEQ = "=ACMGRSVTWYHKDBN"

    def _parse_bam(self, buf: bytes) -> AlignedSegment:
        (ref_id, pos, l_name, mapq, _bin, n_cig, flag, l_seq, _nref, _npos, _tlen) = struct.unpack_from(
            "<iiBBHHHiiii", buf, 0)
        # htslib's bam_read1 checks: the fields fit the block, the query name is NUL-terminated
        if l_seq < 0 or 32 + l_name + 4 * n_cig + (l_seq + 1) // 2 + l_seq > len(buf):
            raise ValueError("invalid BAM record (its fields exceed its block size)")
        if l_name == 0 or buf[32 + l_name - 1] != 0:
            raise ValueError("invalid BAM record (query name not NUL-terminated)")
        o = 32
        qname = buf[o:o + l_name - 1].decode("latin-1")
        o += l_name
        cig = struct.unpack_from("<%dI" % n_cig, buf, o)
        o += 4 * n_cig
        cigar = [(c & 0xF, c >> 4) for c in cig]
        nb = (l_seq + 1) // 2
        sb = buf[o:o + nb]
        o += nb
        seq = "".join(self._SEQ[b >> 4] + self._SEQ[b & 0xF] for b in sb)[:l_seq] if l_seq else None
        qb = buf[o:o + l_seq]
        o += l_seq
        qual = None if (l_seq == 0 or qb[0] == 0xFF) else "".join(chr(q + 33) for q in qb)
        tags = []
        while o < len(buf):
            tg = buf[o:o + 2].decode("latin-1")
            typ = chr(buf[o + 2])
            o += 3
            if typ in "cCsSiI":
                fmt = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I"}[typ]
                v, = struct.unpack_from(fmt, buf, o)
                o += struct.calcsize(fmt)
            elif typ == "f":
                v, = struct.unpack_from("<f", buf, o)
                o += 4
            elif typ == "A":
                v = chr(buf[o])
                o += 1
            elif typ in "ZH":
                e = buf.index(b"\0", o)
                v = buf[o:e].decode("latin-1")
                o = e + 1
            elif typ == "B":
                sub = chr(buf[o])
                cnt, = struct.unpack_from("<i", buf, o + 1)
                fmt = _B_CODES[sub]
                v = array.array(fmt, struct.unpack_from("<%d%s" % (cnt, fmt), buf, o + 5))
                o += 5 + cnt * struct.calcsize(fmt)
            else:
                raise ValueError("bad BAM tag type %r" % typ)
            tags.append((tg, v))
        return AlignedSegment(qname, flag, ref_id, pos, mapq, cigar, seq, qual, tags)

    # ------------------------------------------------------------------ api
    def __iter__(self) -> Iterator[AlignedSegment]:
        if self._bam:
            while True:
                try:
                    n, = struct.unpack("<i", self._read(4, at_record=True))
                except EOFError:
                    return
                buf = self._read(n)
                try:
                    rec = self._parse_bam(buf)
                except (struct.error, IndexError, KeyError, UnicodeDecodeError) as ex:
                    raise ValueError("corrupt BAM record: %s" % ex)
                yield rec
        else:
            if self._pending is not None:
                line, self._pending = self._pending, None
                if line.strip():
                    yield self._parse_sam(line)
            for line in self._fh:
                if line.strip():
                    yield self._parse_sam(line)

    def getrname(self, tid: int) -> str:
        return self.references[tid]

    def close(self):
        try:
            self._fh.close()
        finally:
            if self._raw is not sys.stdin.buffer:
                self._raw.close()


def sam_line(rec: AlignedSegment, references: List[str]) -> str:
    """Format a record back to SAM text (used by tests and the -B writer)."""
    cig = "".join("%d%s" % (n, "MIDNSHP=X"[op]) for op, n in rec.cigar) or "*"
    tags = []
    for t, v in rec.tags:
        if isinstance(v, int):
            tags.append("%s:i:%d" % (t, v))
        elif isinstance(v, float):
            tags.append("%s:f:%.9g" % (t, v))
        elif isinstance(v, array.array):
            sub = {c: k for k, c in _B_CODES.items()}[v.typecode]
            tags.append("%s:B:%s" % (t, ",".join([sub] + ["%.9g" % x if sub == "f" else "%d" % x for x in v])))
        else:
            tags.append("%s:Z:%s" % (t, v))
    return "\t".join([rec.qname, str(rec.flag), references[rec.tid] if rec.tid >= 0 else "*", str(rec.pos + 1),
                      str(rec.mapq), cig, "*", "0", "0", rec.seq or "*", rec.qual or "*"] + tags)
