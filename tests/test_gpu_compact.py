"""The device packer of the compact result forms (fc2_result_compact_launch) where it must escape.
test_gpu_fullsize.py runs it on the 50M-pair bench batch, whose words all fit (0 escapes); here:
(a) the packer's words and escapes equal the numpy restatement of the rule (tests/test_compact_results.py)
word for word on synthetic result words of every shape, escapes included (errors, x > 125 / 254,
n_ties > 16 / 255, dist and ov past their fields); (b) real scan results with many escapes (long
reads, -d 6) expand back bit for bit; (c) an escape list longer than its slots is reported, and the
expansion refuses the truncated list instead of returning wrong words."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from synth_small import load_genome, make_spans
from test_compact_results import pack, sample_words

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from find_circ2_amd import CompactResults, Options, compact, expand  # noqa: E402
from find_circ2_amd import _native as N  # noqa: E402
from test_gpu_parity import genome, run_spans  # noqa: E402


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _device_form(opt, words8, width, cap=0):
    dev = _dev()
    d = torch.from_numpy(words8.astype(np.int64)).to(dev)
    c = compact(opt, d, len(words8), into=CompactResults(len(words8), dev, cap=cap, width=width))
    torch.cuda.synchronize(dev)
    k = int(c.count.item())
    esc = c.esc.cpu().numpy().view(N.ESCAPE_DTYPE)[:min(k, c.cap)]
    return c.words[:len(words8)].cpu().numpy(), np.sort(esc, order="index"), k, c.cap


@pytest.mark.parametrize("width", [2, 4])
def test_device_words_equal_the_restated_rule(width):
    w = sample_words(400_003, seed=17).astype(np.int64)
    got, esc, k, cap = _device_form(Options(), w, width, cap=len(w))
    exp, exp_esc = pack(w.view(np.uint64), width)
    assert np.array_equal(got.view(exp.dtype), exp)
    assert k == len(exp_esc) > 1000
    assert np.array_equal(esc["index"], exp_esc["index"])
    assert np.array_equal(esc["result"].view(np.int64), exp_esc["result"].view(np.int64))
    assert np.array_equal(expand(Options(), got, esc), w)


@pytest.mark.parametrize("width", [2, 4])
def test_scan_results_with_escapes_expand_back(width):
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    opt = Options(maxdist=6, margin=0)
    spans = make_spans(load_genome(path), 6000, seed=606, asize=opt.asize, L=(60, 300), p_readN=0.05)
    b, out = run_spans(opt, genome(path), spans)
    res = out.results[:b.n].cpu().numpy()
    got, esc, k, cap = _device_form(opt, res, width)
    assert k <= cap
    if width == 2:
        assert k > 100                              # x > 125 and dist > 3 are common here
    assert np.array_equal(expand(opt, got, esc), res)


def test_escape_overflow_is_reported():
    w = sample_words(50_000, seed=23).astype(np.int64)
    got, esc, k, cap = _device_form(Options(), w, 2, cap=16)
    assert cap == 16 and k > cap
    with pytest.raises(Exception):
        expand(Options(), got, esc)


# --- the scan writing the compact form itself (fc2_bp_scan_compact_launch) ------------------------

def _compact_scan(opt, g, b, width, cap, host):
    """Run scan_compact into device memory or into page-locked host memory (through its device
    address); return words, escapes sorted by index, the moved count, and the device counter after."""
    import mmap
    from find_circ2_amd.hotpath import host_device_pointer, scan_compact
    dev = _dev()
    n = b.n
    wbytes = (width * n + 63) // 64 * 64
    size = wbytes + 16 * (cap + 1)
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)
    if host:
        mm = mmap.mmap(-1, size)
        buf = np.frombuffer(mm, np.uint8)
        buf[:] = 0xA5
        N.check(N.lib().fc2_host_register(buf.ctypes.data, size))
        base = host_device_pointer(buf.ctypes.data)
    else:
        dbuf = torch.full((size,), 0xA5, dtype=torch.uint8, device=dev)
        base = dbuf.data_ptr()
    try:
        scan_compact(opt, g, b, base, width, base + wbytes, cap, ctr.data_ptr(), base + wbytes + 16 * cap)
        torch.cuda.synchronize(dev)
        raw = buf.copy() if host else dbuf.cpu().numpy()
    finally:
        if host:
            N.lib().fc2_host_unregister(buf.ctypes.data)
            del buf
            mm.close()
    words = raw[:width * n].view(np.uint16 if width == 2 else np.uint32)
    k = int(raw[wbytes + 16 * cap:wbytes + 16 * cap + 4].view(np.int32)[0])
    esc = raw[wbytes:wbytes + 16 * cap].view(N.ESCAPE_DTYPE)[:min(k, cap)]
    return words, np.sort(esc, order="index"), k, int(ctr.item())


@pytest.mark.parametrize("host", [False, True], ids=["device_memory", "host_memory"])
@pytest.mark.parametrize("width", [2, 4])
def test_compact_scan_equals_pack_of_the_scan(width, host):
    """The scan's own compact epilogue writes the words and escapes the packer writes from the
    8-byte scan (escape-heavy spans: long reads, -d 6), into device memory or straight into
    page-locked host memory; the count moves to its slot and the device counter is zero again."""
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    opt = Options(maxdist=6, margin=0)
    spans = make_spans(load_genome(path), 6000, seed=606, asize=opt.asize, L=(60, 300), p_readN=0.05)
    g = genome(path)
    b, out = run_spans(opt, g, spans)
    assert b.m_bytepath == 0
    res = out.results[:b.n].cpu().numpy()
    exp_words, exp_esc, exp_k, _ = _device_form(opt, res, width, cap=b.n)
    words, esc, k, ctr = _compact_scan(opt, g, b, width, b.n, host)
    assert ctr == 0
    assert k == exp_k and (width == 4 or k > 100)
    assert np.array_equal(words, exp_words.view(words.dtype))
    assert np.array_equal(esc["index"], exp_esc["index"])
    assert np.array_equal(esc["result"].view(np.int64), exp_esc["result"].view(np.int64))
    assert np.array_equal(expand(opt, words, esc), res)


def test_compact_scan_hg19_shaped_batch_and_refusals():
    """A read-order batch on the hg19-shaped genome (the staged headline form): the 2-byte words from
    the scan equal the packer's, 0 escapes; --non-canonical / --all-hits are refused."""
    from find_circ2_amd import Genome, PairBatch, SynthConfig, scan, sq_table
    from find_circ2_amd.hotpath import scan_compact
    dev = _dev()
    names, sizes = sq_table(os.path.join(GOLDEN, "test_norm.sam"))
    g = Genome.synthetic(names, sizes, seed=4711, device=dev)
    opt = Options()
    b = PairBatch.synthetic(opt, g, 2_000_000, SynthConfig(seed=77, span_max=20000))
    res = scan(opt, g, b).results[:b.n]
    torch.cuda.synchronize(dev)
    exp_words, exp_esc, exp_k, _ = _device_form(opt, res.cpu().numpy(), 2)
    words, esc, k, ctr = _compact_scan(opt, g, b, 2, 4096, host=True)
    assert k == exp_k == 0 and ctr == 0
    assert np.array_equal(words, exp_words.view(words.dtype))
    ctr_t = torch.zeros(1, dtype=torch.int32, device=dev)
    buf = torch.empty(2 * b.n, dtype=torch.uint8, device=dev)
    for bad in (Options(noncanonical=True), Options(allhits=True)):
        with pytest.raises(Exception):
            scan_compact(bad, g, b, buf.data_ptr(), 2, 0, 0, ctr_t.data_ptr())


@pytest.mark.parametrize("file_seg", [False, True], ids=["shm", "file"])
@pytest.mark.parametrize("width", [2, 4])
def test_sharded_zero_copy_merge_with_escapes(width, file_seg, monkeypatch):
    """bench.py's configs[3] merge on escape-heavy pairs (long reads, -d 6): sub-batch views of one
    batch dealt to 3 "ranks" (shard.round_bounds / my_bounds) each scan straight into ONE page-locked
    SharedCompactResults through its device address (words at the batch's input offset, escapes into
    the batch's slots with batch-relative indices, the count into its slot); merged() -- escapes()
    adding each batch's start back, then fc2_result_expand -- equals the 8-byte scan of the whole
    batch word for word.  file_seg: the buffer in a shared file mapping (a node whose /dev/shm has no
    room, shard._segment), page-locked and written by the GPU the same way."""
    from find_circ2_amd import shard
    from find_circ2_amd.hotpath import host_device_pointer, scan_compact
    from find_circ2_amd.shard import SharedCompactResults, my_bounds, round_bounds
    if file_seg:
        monkeypatch.setattr(shard, "SHM_DIR", "/nonexistent")
    dev = _dev()
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    opt = Options(maxdist=6, margin=0)
    spans = make_spans(load_genome(path), 12000, seed=909, asize=opt.asize, L=(60, 300), p_readN=0.05)
    g = genome(path)
    b, out = run_spans(opt, g, spans)
    assert b.m_bytepath == 0
    ref = out.results[:b.n].cpu().numpy()
    ws = 3
    bounds = round_bounds(b.n, ws, per_rank=2, align=512, tail=2)
    cap = 4096
    m = SharedCompactResults(b.n, bounds, cap, create=True, pin=True, width=width)
    assert m.name.startswith("file:") == file_seg
    try:
        m.array[:] = 0x5A                                          # poison: every word must be written
        zdev = host_device_pointer(m.array.ctypes.data)
        zblk = 16 * (cap + 1)
        ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        n_esc = 0
        for rank in range(ws):
            for k, lo, hi in my_bounds(bounds, rank, ws):
                eb = zdev + m._w_bytes + k * zblk
                scan_compact(opt, g, b.sub(lo, hi), zdev + width * lo, width, eb, cap, ctr.data_ptr(), eb + 16 * cap)
        torch.cuda.synchronize(dev)
        n_esc = int(m.esc_count.sum())
        assert (m.esc_count <= cap).all()
        if width == 2:
            assert n_esc > 100 and (m.esc_count[:len(bounds)] > 0).sum() >= 3
        assert np.array_equal(m.merged(opt), ref)
    finally:
        m.close()


@pytest.mark.parametrize("width", [2, 4])
def test_compact_launch_marks_byte_path_pairs(width):
    """fc2_bp_scan_compact_launch takes no byte-path pairs (fc2_bp.h); a C host that passes some
    gets the escape word without an escape record for each of them, so fc2_result_expand fails
    (FC2_E_FORMAT) instead of decoding whatever the word held before."""
    import ctypes
    dev = _dev()
    path = os.path.join(GOLDEN, "CDR1as_locus.fa")
    opt = Options()
    spans = make_spans(load_genome(path), 600, seed=5, asize=opt.asize, L=(60, 120))
    reads = [s.read_part for s in spans]
    reads[17] = reads[17][:30] + b"R" + reads[17][31:]           # an IUPAC byte: byte-exact path
    from find_circ2_amd import PairBatch
    g = genome(path)
    flags = [(N.PAIR_BACKSPLICE if s.is_backsplice else 0) for s in spans]
    b = PairBatch.pack(opt, g, reads, [s.a_pos for s in spans], [s.b_aend for s in spans],
                       [g.chrom_index_or_missing(s.chrom) for s in spans], flags)
    assert b.m_bytepath >= 1
    n = b.n
    words = torch.full((n * width // 2 + 8,), 0x2A2A, dtype=torch.int16, device=dev)   # stale contents
    esc = torch.zeros(16 * 64, dtype=torch.uint8, device=dev)
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)
    co = N.CompactOut(width, 64, words.data_ptr(), esc.data_ptr(), ctr.data_ptr(), None)
    p, gv, bv = opt.params(), g.view(), b.view()
    N.check(N.lib().fc2_bp_scan_compact_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv),
                                               ctypes.byref(co), torch.cuda.current_stream(dev).cuda_stream))
    torch.cuda.synchronize(dev)
    k = int(ctr.item())
    w = words.cpu().numpy().view(np.uint16 if width == 2 else np.uint32)[:n]
    e = esc.cpu().numpy().view(N.ESCAPE_DTYPE)[:min(k, 64)]
    bp = np.nonzero(b.host_pairs["flags"] & N.PAIR_BYTEPATH)[0]
    marker = N.R16_ESCAPE if width == 2 else N.R32_ESCAPE
    assert (w[bp] == marker).all()
    with pytest.raises(N.Fc2Error) as ei:
        expand(opt, w, e)
    assert ei.value.code == N.FC2_E_FORMAT
