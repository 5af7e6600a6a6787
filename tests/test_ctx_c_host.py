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
