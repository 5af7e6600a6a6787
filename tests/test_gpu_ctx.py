"""The per-device context (include/fc2_ctx.h): the torch-free C ABI form of the drop-in boundary
(SURVEY.md §8(b)).  Its genome load and batch pipeline must give, word for word, the results of the
Python host layer (PairBatch.pack + scan, itself checked against the oracle in test_gpu_parity.py),
and the oracle's answers: options, --all-hits tie masks, the byte path (IUPAC / CRLF / irregular
FASTA, very long reads), the dummy genome, reuse of one context over batches of different shapes."""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN
from gpu_helpers import assert_same, gpu_arrays, oracle_arrays
from synth_small import load_genome, make_spans

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import Genome, Options  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402
from test_gpu_parity import OPTS, WEIRD, genome, oracle_spans, run_spans  # noqa: E402


class Ctx:
    def __init__(self, path=None, prepack=False):
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
        self.L = N.lib()
        self.c = ctypes.c_void_p()
        self.fa = ctypes.c_void_p()
        if path:
            N.check(self.L.fc2_fasta_open(path.encode(), 0, ctypes.byref(self.fa)))
            if prepack:                 # the CLI's start-up: planes packed before (beside) HIP init
                N.check(self.L.fc2_fasta_prepack(self.fa, 0))
        N.check(self.L.fc2_ctx_create(0, ctypes.byref(self.c)))
        self.check(self.L.fc2_ctx_genome_load(self.c, self.fa if path else None, 0))

    def check(self, rc):
        if rc != N.FC2_OK:
            raise N.Fc2Error(rc, self.L.fc2_ctx_last_error(self.c).decode())

    def chrom(self, name):
        return self.L.fc2_fasta_find(self.fa, name.encode()) & 0xFFFFFFFF if self.fa else 0

    def scan(self, opt, spans, tw=0):
        reads = [s.read_part for s in spans]
        n = len(reads)
        off = np.zeros(n, np.uint64)
        lens = np.array([len(r) for r in reads], np.int64)
        if n:
            off[1:] = np.cumsum(lens[:-1])
        buf = np.frombuffer(b"".join(reads) + b"\0" * 16, np.uint8)
        pairs = np.zeros(n, N.PAIR_DTYPE)
        pairs["a_pos"] = [s.a_pos for s in spans]
        pairs["b_aend"] = [s.b_aend for s in spans]
        pairs["chrom"] = [self.chrom(s.chrom) for s in spans]
        pairs["read_len"] = lens
        pairs["flags"] = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) | (N.PAIR_PRIMARY_REV if s.primary_reverse else 0)
                          for s in spans]
        res = np.zeros(max(n, 1), np.int64)
        tm = np.zeros(max(tw * n, 1), np.int64) if opt.allhits else None
        p = opt.params()
        self.check(self.L.fc2_ctx_scan_async(self.c, ctypes.byref(p), n, buf.ctypes.data, off.ctypes.data,
                                             pairs.ctypes.data, res.ctypes.data,
                                             tm.ctypes.data if tm is not None else None, tw, 0))
        self.check(self.L.fc2_ctx_sync(self.c))
        return res[:n], (tm[:tw * n] if tm is not None else None)

    def close(self):
        self.L.fc2_ctx_destroy(self.c)
        if self.fa:
            self.L.fc2_fasta_close(self.fa)


def _compare(opt, path, g, spans, ctx, label):
    b, out = run_spans(opt, g, spans)
    res, tm = ctx.scan(opt, spans, b.tw)
    assert np.array_equal(res, out.results[:b.n].cpu().numpy()), label + ": results differ from the Python path"
    if opt.allhits:
        assert np.array_equal(tm, out.tiemask[:b.tw * b.stride].cpu().numpy()), label + ": tie masks differ"
    if path is not None:
        r = oracle_spans(opt, path, spans, g.names)
        return assert_same(gpu_arrays(opt, b.host_pairs, res.view(N.RESULT_DTYPE)), oracle_arrays(r), label=label)
    return 0


@pytest.mark.parametrize("prepack", [False, True], ids=["pack", "prepacked"])
@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
def test_ctx_equals_python_path_and_oracle(fa, prepack):
    path = os.path.join(GOLDEN, fa)
    g = genome(path)
    ctx = Ctx(path, prepack=prepack)
    try:
        gen = load_genome(path)
        for oi in (0, 1, 3, 5, 6, 8):
            opt = Options(**OPTS[oi])
            # batches of different sizes and read lengths through ONE context (its buffers grow)
            n, L = ((500, (40, 120)), (3000, (40, 300)), (1200, (30, 90)))[oi % 3]
            spans = make_spans(gen, n, seed=8100 + oi, asize=opt.asize, L=L, p_readN=0.1)
            assert _compare(opt, path, g, spans, ctx, "%s %s" % (fa, OPTS[oi])) > 10
    finally:
        ctx.close()


@pytest.mark.parametrize("prepack", [False, True], ids=["pack", "prepacked"])
def test_ctx_byte_path_and_long_reads(tmp_path, prepack):
    path = str(tmp_path / "weird.fa")
    open(path, "wb").write(b"".join(WEIRD.replace(b">c", b">r%dc" % k) for k in range(3)))
    g = Genome.from_fasta(path, device="cuda:0")
    ctx = Ctx(path, prepack=prepack)
    try:
        gen = load_genome(path)
        for o in (dict(asize=6, margin=1, maxdist=3), dict(asize=6, margin=2, maxdist=2, allhits=True, noncanonical=True)):
            opt = Options(**o)
            spans = make_spans(gen, 1500, seed=77, asize=opt.asize, L=(12, 60), p_edge=0.3, p_readN=0.2)
            _compare(opt, path, g, spans, ctx, "weird " + str(o))
    finally:
        ctx.close()
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    ctx = Ctx(path)
    try:
        spans = []
        for L in (20, 26, 27, 129, 257, 520, 524, 1000):
            spans += make_spans(load_genome(path), 10, seed=L, L=(L, L), asize=15, p_short=0.0)
        _compare(Options(), path, genome(path), spans, ctx, "edge lengths")
    finally:
        ctx.close()


def test_ctx_dummy_genome_and_empty_batch():
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    g = Genome.dummy_genome(device="cuda:0")
    ctx = Ctx(None)
    try:
        spans = make_spans(load_genome(path), 300, seed=3, p_readN=0.0)
        for s in spans[:100]:
            s.read_part = b"A" * 13 + b"N" * (len(s.read_part) - 26) + b"T" * 13
        for o in (dict(), dict(noncanonical=True, maxdist=5)):
            _compare(Options(**o), None, g, spans, ctx, "dummy " + str(o))
        res, _ = ctx.scan(Options(), [])
        assert len(res) == 0
    finally:
        ctx.close()


def test_ctx_refuses_a_second_batch_before_sync():
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    ctx = Ctx(path)
    try:
        L = ctx.L
        spans = make_spans(load_genome(path), 50, seed=1)
        opt = Options()
        reads = np.frombuffer(b"".join(s.read_part for s in spans) + b"\0" * 16, np.uint8)
        off = np.cumsum([0] + [len(s.read_part) for s in spans[:-1]]).astype(np.uint64)
        pairs = np.zeros(len(spans), N.PAIR_DTYPE)
        pairs["read_len"] = [len(s.read_part) for s in spans]
        pairs["a_pos"] = [s.a_pos for s in spans]
        pairs["b_aend"] = [s.b_aend for s in spans]
        res = np.zeros(len(spans), np.int64)
        p = opt.params()
        args = (ctypes.byref(p), len(spans), reads.ctypes.data, off.ctypes.data, pairs.ctypes.data, res.ctypes.data,
                None, 0, 0)
        assert L.fc2_ctx_scan_async(ctx.c, *args) == N.FC2_OK
        assert L.fc2_ctx_scan_async(ctx.c, *args) == N.FC2_E_PARAM
        assert b"not synced" in L.fc2_ctx_last_error(ctx.c)
        assert L.fc2_ctx_sync(ctx.c) == N.FC2_OK
        assert (res != 0).all()
        gv = N.GenomeView()
        assert L.fc2_ctx_genome_view(ctx.c, ctypes.byref(gv)) == N.FC2_OK
        assert gv.wt and gv.units and gv.n_chrom == 1
        assert L.fc2_ctx_stream(ctx.c)
    finally:
        ctx.close()


@pytest.mark.parametrize("o", [dict(), dict(allhits=True, noncanonical=True)])
@pytest.mark.parametrize("background", [False, True])
def test_ctxpipe_round_robin_equals_python_path(o, background):
    """ctxpipe.CtxPipeline (the CLI's evaluator: a context + sibling contexts sharing its resident
    genome, chunks dealt round-robin, results in submission order; with background=True chunks
    submitted while the genome is still being built are dispatched in order once it is ready):
    every chunk's words and tie masks equal the Python layer's scan of the same pairs."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd.ctxpipe import CtxPipeline, FastaGenome
    opt = Options(**o)
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    g = genome(path)
    fg = FastaGenome(path, write_index=False)
    pipe = CtxPipeline(fg, opt, devices=["cuda:0", "cuda:0"], per_device=2, background=background)
    try:
        assert pipe.n_ctx == 4 and pipe.depth == 16
        chunks, tickets = [], []
        for k in range(11):
            spans = make_spans(load_genome(path), 300 + 37 * k, seed=900 + k, L=(40, 700), p_readN=0.05)
            reads = [s.read_part for s in spans]
            off = np.zeros(len(reads), np.uint64)
            off[1:] = np.cumsum([len(r) for r in reads[:-1]])
            buf = np.frombuffer(b"".join(reads) + b"\0" * 16, np.uint8)
            pairs = np.zeros(len(reads), N.PAIR_DTYPE)
            pairs["a_pos"] = [s.a_pos for s in spans]
            pairs["b_aend"] = [s.b_aend for s in spans]
            pairs["chrom"] = [g.chrom_index(s.chrom) for s in spans]
            pairs["read_len"] = [len(r) for r in reads]
            pairs["flags"] = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) |
                              (N.PAIR_PRIMARY_REV if s.primary_reverse else 0) for s in spans]
            chunks.append((spans, buf))
            tickets.append(pipe.submit(buf.ctypes.data, off, pairs))
        for (spans, buf), t in zip(chunks, tickets):
            res, tm = pipe.result(t)
            b, out = run_spans(opt, g, spans)
            assert np.array_equal(res, out.host(b.n).view(np.int64)), "words"
            if opt.allhits:
                ref = out.tiemask[:b.tw * b.stride].cpu().numpy().view(np.uint64).reshape(b.tw, b.stride)
                assert np.array_equal(tm, ref[:tm.shape[0], :b.n]), "tie mask"
    finally:
        pipe.close()
        fg.close()
