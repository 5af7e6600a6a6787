"""spliced_reads.fastq.gz writer: parallel gzip members decode to the written text."""
import gzip
import zlib

import pytest

from find_circ2_amd.gzout import ParallelGzipWriter


@pytest.mark.parametrize("piece,threads", [(1 << 22, 0), (997, 3), (1, 2)])
def test_members_decode_to_text(tmp_path, piece, threads):
    p = str(tmp_path / "r.fastq.gz")
    w = ParallelGzipWriter(p, piece=piece, threads=threads)
    text = []
    for i in range(3000):
        s = "@read%d junc_%d FLAG\nACGTN%d\n+read%d\nIIII#\n" % (i, i % 7, i, i)
        w.write(s)
        text.append(s)
    w.close()
    assert gzip.open(p, "rt").read() == "".join(text)
    raw = open(p, "rb").read()
    assert raw[:2] == b"\x1f\x8b"
    d = zlib.decompressobj(16 + zlib.MAX_WBITS)          # first member alone is a full gzip stream
    assert d.decompress(raw)


def test_empty_file_is_valid_gzip(tmp_path):
    p = str(tmp_path / "e.gz")
    ParallelGzipWriter(p).close()
    assert gzip.open(p, "rt").read() == ""
