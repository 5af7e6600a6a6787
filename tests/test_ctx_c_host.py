"""A C program that binds only include/fc2_ctx.h (tests/c/ctx_host.c): compiled
with gcc against the shipped libfc2.so; on the GPU its results equal the Python layer's word for
word, without PyTorch in its process; without a GPU it fails cleanly with the library's message."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from find_circ2_amd import _native as N
from synth_small import load_genome, make_spans

LIBDIR = os.path.join(ROOT, "find_circ2_amd")


@pytest.fixture(scope="module")
def ctx_host(tmp_path_factory):
    N.build()
    exe = str(tmp_path_factory.mktemp("c") / "ctx_host")
    r = subprocess.run(["gcc", "-O1", "-Wall", "-Werror", "-std=c11", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "c", "ctx_host.c"), "-o", exe, "-L", LIBDIR, "-lfc2",
                        "-Wl,-rpath," + LIBDIR, "-Wl,--allow-shlib-undefined"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    assert r.returncode == 0, r.stderr.decode()
    return exe


def _batch(path, spans, chrom_of):
    reads = [s.read_part for s in spans]
    n = len(reads)
    off = np.zeros(n, np.uint64)
    lens = np.array([len(x) for x in reads], np.int64)
    if n:
        off[1:] = np.cumsum(lens[:-1])
    pairs = np.zeros(n, N.PAIR_DTYPE)
    pairs["a_pos"] = [s.a_pos for s in spans]
    pairs["b_aend"] = [s.b_aend for s in spans]
    pairs["chrom"] = [chrom_of(s.chrom) for s in spans]
    pairs["read_len"] = lens
    pairs["flags"] = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
                      for s in spans]
    with open(path, "wb") as fh:
        fh.write(np.uint64(n).tobytes() + pairs.tobytes() + off.tobytes() + b"".join(reads))
    return pairs


def test_c_host_builds_and_fails_cleanly_without_a_gpu(ctx_host, tmp_path):
    import ctypes
    c = ctypes.c_int(0)
    N.lib().fc2_device_count(ctypes.byref(c))
    if c.value:
        pytest.skip("a GPU is visible (the GPU test covers this host)")
    fa = os.path.join(GOLDEN, "CDR1as_locus.fa")
    spans = make_spans(load_genome(fa), 20, seed=5)
    _batch(str(tmp_path / "b.bin"), spans, lambda name: 0)
    r = subprocess.run([ctx_host, fa, str(tmp_path / "b.bin"), str(tmp_path / "r.bin"), "15", "2", "2"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert r.returncode == 2 and b"fc2_ctx_create" in r.stderr, r.stderr


@pytest.mark.gpu
def test_c_host_equals_python_layer(ctx_host, tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import Genome, Options, PairBatch, scan
    for fa in ("CDR1as_locus.fa", "test_ref.fa"):
        path = os.path.join(GOLDEN, fa)
        g = Genome.from_fasta(path, device="cuda:0")
        spans = make_spans(load_genome(path), 2500, seed=31, L=(40, 260), p_readN=0.1)
        pairs = _batch(str(tmp_path / "b.bin"), spans, g.chrom_index_or_missing)
        opt = Options()
        b = PairBatch.pack(opt, g, [s.read_part for s in spans], pairs["a_pos"], pairs["b_aend"], pairs["chrom"],
                           pairs["flags"])
        exp = scan(opt, g, b).results[:b.n].cpu().numpy()
        r = subprocess.run([ctx_host, path, str(tmp_path / "b.bin"), str(tmp_path / "r.bin"), "15", "2", "2"],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
        assert r.returncode == 0, r.stderr.decode()
        got = np.fromfile(str(tmp_path / "r.bin"), np.int64)
        assert np.array_equal(got, exp), fa
        assert ((got & 0xFFFF) != 0xFFFF).sum() > 100


def _build(tmp_path_factory, src, name):
    exe = str(tmp_path_factory.mktemp("c") / name)
    r = subprocess.run(["gcc", "-O1", "-Wall", "-Werror", "-std=c11", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "c", src), "-o", exe, "-L", LIBDIR, "-lfc2",
                        "-Wl,-rpath," + LIBDIR, "-Wl,--allow-shlib-undefined"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    assert r.returncode == 0, r.stderr.decode()
    return exe


@pytest.fixture(scope="module")
def findcirc_host(tmp_path_factory):
    N.build()
    return _build(tmp_path_factory, "findcirc_host.c", "findcirc_host")


def test_c_findcirc_builds_and_fails_cleanly_without_a_gpu(findcirc_host, tmp_path):
    import ctypes
    c = ctypes.c_int(0)
    N.lib().fc2_device_count(ctypes.byref(c))
    if c.value:
        pytest.skip("a GPU is visible (the GPU test covers this program)")
    from test_ingest import _mixed_sam
    sam = str(tmp_path / "in.sam")
    fa = _mixed_sam(sam, 50, seed=3)
    r = subprocess.run([findcirc_host, "-G", fa, "-o", str(tmp_path / "out"), sam], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=120)
    assert r.returncode == 2 and b"fc2_ctx_create" in r.stderr, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("genome", ["fasta", "folder", "long_reads"])
def test_c_findcirc_equals_the_python_cli(findcirc_host, tmp_path, genome):
    """The whole read loop and the search driven from C (no Python in the process) write the
    Python CLI's files: both BED tables, multi_events.tsv and spliced_reads.fastq (decompressed).
    With -G naming a folder, both run in GenomeAccessor's dummy mode (find_circ.py:338-345); with
    read parts over 32767 bases the C host evaluates the long pairs (fc2_ctx_scan_long,
    fc2_caller_submit_long)."""
    import gzip
    import sys
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from test_ingest import _mixed_sam
    sam = str(tmp_path / "in.sam")
    if genome == "long_reads":
        from test_read_limits import _long_read_genome, _long_reads, _sam_of
        g = _long_read_genome(36000)
        reads = _long_reads(g, 36000)                 # (plants the splice signals into g)
        fa = str(tmp_path / "g.fa")
        with open(fa, "w") as f:
            for c, sq in g.items():
                t = sq.decode()
                f.write(">%s\n" % c + "".join(t[i:i + 60] + "\n" for i in range(0, len(t), 60)))
        open(sam, "w").write(_sam_of(g, reads))
    else:
        fa = _mixed_sam(sam, 3000, seed=4711)
    if genome == "folder":
        fa = str(tmp_path / "genome_folder")
        os.makedirs(fa)
    py_out, c_out = str(tmp_path / "py"), str(tmp_path / "c")
    r = subprocess.run([sys.executable, "-m", "find_circ2_amd.cli", "-G", fa, "-o", py_out, "-n", "cx", "-q", sam],
                       cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    r = subprocess.run([findcirc_host, "-G", fa, "-o", c_out, "-n", "cx", sam], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    for f in ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv"):
        a, b = open(os.path.join(py_out, f), "rb").read(), open(os.path.join(c_out, f), "rb").read()
        assert a == b, f
    circ = open(os.path.join(c_out, "circ_splice_sites.bed")).read().splitlines()
    if genome == "folder":
        assert b"Switching to dummy mode" in r.stderr
        assert len(circ) == 1                         # the header: all-N windows never hold a GT/AG signal
        return
    assert len(circ) > (2 if genome == "long_reads" else 10)
    a = gzip.open(os.path.join(py_out, "spliced_reads.fastq.gz")).read()
    b = gzip.open(os.path.join(c_out, "spliced_reads.fastq.gz")).read()
    assert a == b and len(a) > 1000
