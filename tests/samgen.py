"""Write bwa-mem-shaped SAM/BAM for test reads (no aligner in this image).

Per read: the longest exact segment is the primary record (full SEQ, soft
clips, flag 0/16), every other segment a supplementary record (flag 2048 |
strand, hard clips, SEQ = aligned part), tags AS (= segment length) and NM,
like bwa mem's output shape in test_data/test_norm.sam.
"""
import gzip
import struct

from bwa_emul import revcomp, segment_read


def records_for_read(qname, read, genome, min_len=12, flag_extra=0, xs=None):
    best = None
    for rev in (False, True):
        seq = revcomp(read) if rev else read.upper()
        segs = segment_read(seq, genome, min_len)
        cov = sum(s.q_end - s.q_start for s in segs)
        if best is None or cov > best[2]:
            best = (rev, seq, cov, segs)
    rev, seq, _, segs = best
    L = len(seq)
    if not segs:
        return [dict(qname=qname, flag=4 | flag_extra, rname="*", pos=0, cigar="*", seq=seq, qual="I" * L, tags=[])]
    prim = max(range(len(segs)), key=lambda k: segs[k].q_end - segs[k].q_start)
    out = []
    strand = 16 if rev else 0
    for k in [prim] + [k for k in range(len(segs)) if k != prim]:
        s = segs[k]
        clip = "S" if k == prim else "H"
        cig = ("%d%s" % (s.q_start, clip) if s.q_start else "") + "%dM" % (s.q_end - s.q_start) + \
              ("%d%s" % (L - s.q_end, clip) if L - s.q_end else "")
        tags = [("NM", "i", 0), ("AS", "i", s.q_end - s.q_start)]
        if xs is not None:
            tags.append(("XS", "i", xs))
        out.append(dict(qname=qname, flag=strand | flag_extra | (0 if k == prim else 2048), rname=s.chrom,
                        pos=s.pos + 1, cigar=cig, seq=seq if k == prim else seq[s.q_start:s.q_end],
                        qual=("I" * L) if k == prim else "*", tags=tags))
    return out


def sam_text(genome, reads, **kw):
    lines = ["@HD\tVN:1.5\tSO:unsorted"]
    for name, g in genome.items():
        lines.append("@SQ\tSN:%s\tLN:%d" % (name, len(g)))
    for qname, read in reads:
        for r in records_for_read(qname, read, genome, **kw):
            tags = ["%s:%s:%s" % t for t in r["tags"]]
            lines.append("\t".join([r["qname"], str(r["flag"]), r["rname"], str(r["pos"]), "60" if r["rname"] != "*"
                                    else "0", r["cigar"], "*", "0", "0", r["seq"], r["qual"]] + tags))
    return "\n".join(lines) + "\n"


_SEQ_CODE = {c: i for i, c in enumerate("=ACMGRSVTWYHKDBN")}
_OPS = {c: i for i, c in enumerate("MIDNSHP=X")}


def bgzf_compress(data: bytes, block: int = 65280, level: int = 6) -> bytes:
    """BGZF (SAM/BAM spec 4.1): gzip members of <= 64 KiB, compressed size in a 'BC' extra
    field, followed by the 28-byte empty EOF block."""
    import zlib
    out = bytearray()
    for k in range(0, len(data), block):
        chunk = data[k:k + block]
        co = zlib.compressobj(level, zlib.DEFLATED, -15)
        cdata = co.compress(chunk) + co.flush()
        bsize = 18 + len(cdata) + 8
        out += b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", bsize - 1)
        out += cdata + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


def sam_to_bam(sam: str, path: str, bgzf: bool = True, compress: str = ""):
    """Minimal BAM writer: BGZF blocks (as samtools writes them) or, with ``bgzf=False``,
    one plain gzip member (some tools do; readers must accept both).  ``compress="none"``
    writes the bare BAM bytes (no gzip framing at all; htslib reads that too)."""
    compress = compress or ("bgzf" if bgzf else "gzip")
    import re
    refs, recs = [], []
    for line in sam.splitlines():
        if line.startswith("@SQ"):
            d = dict(kv.split(":", 1) for kv in line.split("\t")[1:])
            refs.append((d["SN"], int(d["LN"])))
        elif line and not line.startswith("@"):
            recs.append(line.split("\t"))
    text = "\n".join(l for l in sam.splitlines() if l.startswith("@")) + "\n"
    tid = {n: i for i, (n, _) in enumerate(refs)}
    out = bytearray(b"BAM\1")
    out += struct.pack("<i", len(text)) + text.encode()
    out += struct.pack("<i", len(refs))
    for n, ln in refs:
        out += struct.pack("<i", len(n) + 1) + n.encode() + b"\0" + struct.pack("<i", ln)
    for f in recs:
        qn = f[0].encode() + b"\0"
        cig = [(int(n), _OPS[op]) for n, op in re.findall(r"(\d+)([MIDNSHP=X])", f[5])] if f[5] != "*" else []
        seq = f[9] if f[9] != "*" else ""
        sb = bytearray()
        for i in range(0, len(seq), 2):
            a = _SEQ_CODE[seq[i]]
            b = _SEQ_CODE[seq[i + 1]] if i + 1 < len(seq) else 0
            sb.append((a << 4) | b)
        qual = bytes([ord(c) - 33 for c in f[10]]) if f[10] != "*" else b"\xff" * len(seq)
        aux = bytearray()
        for t in f[11:]:
            tg, typ, val = t.split(":", 2)
            if typ == "i":
                aux += tg.encode() + b"i" + struct.pack("<i", int(val))
            elif typ == "f":                                # float32, as htslib stores a SAM 'f' value
                aux += tg.encode() + b"f" + struct.pack("<f", float(val))
            elif typ == "A":
                aux += tg.encode() + b"A" + val.encode()[:1]
            elif typ == "B":
                sub, *vals = val.split(",")
                fmt = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}[sub]
                aux += tg.encode() + b"B" + sub.encode() + struct.pack("<i%d%s" % (len(vals), fmt), len(vals),
                                                                      *[(float if sub == "f" else int)(v) for v in vals])
            else:
                aux += tg.encode() + b"Z" + val.encode() + b"\0"
        body = struct.pack("<iiBBHHHiiii", tid.get(f[2], -1), int(f[3]) - 1, len(qn), int(f[4]), 0, len(cig),
                           int(f[1]), len(seq), -1, -1, 0)
        body += qn + b"".join(struct.pack("<I", (n << 4) | op) for n, op in cig) + bytes(sb) + qual + bytes(aux)
        out += struct.pack("<i", len(body)) + body
    if compress == "bgzf":
        with open(path, "wb") as fh:
            fh.write(bgzf_compress(bytes(out)))
    elif compress == "gzip":
        with gzip.open(path, "wb") as fh:
            fh.write(bytes(out))
    else:
        with open(path, "wb") as fh:
            fh.write(bytes(out))
