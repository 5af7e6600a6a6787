"""BGZF blocks inflated on the GPU (fc2_bgzf_inflate_launch, csrc/fc2_inflate.hip) against zlib: every
DEFLATE form zlib writes (stored, fixed and dynamic Huffman codes, every level and strategy), the
blocks of real BGZF BAMs (fc2_sam_to_bam at level 1, the test BGZF writer at level 6), long and
overlapping matches, empty and full 64-KiB blocks; and damaged payloads, which must end in a status
word (never a fault), the host then checking CRC-32 and size as it does for the CPU inflate."""
import os
import zlib

import numpy as np
import pytest

from conftest import GOLDEN

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SLOT = 65536


def _deflate(data: bytes, level=6, strategy=zlib.Z_DEFAULT_STRATEGY) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    return c.compress(data) + c.flush()


def _run(payloads, sizes, crcs=None):
    """The kernel over payloads (raw DEFLATE) claimed to hold sizes bytes (with CRC-32s crcs, if
    given): (outputs, status)."""
    import ctypes
    from find_circ2_amd import _native as N
    n = len(payloads)
    off, buf = [], bytearray()
    rng = np.random.default_rng(len(payloads))
    for p in payloads:
        buf += bytes(int(rng.integers(0, 4)))          # payloads at every byte alignment
        off.append(len(buf))
        buf += p
    buf += bytes(64)                                    # readable past every payload
    dev = torch.device("cuda:0")
    src = torch.tensor(np.frombuffer(bytes(buf), np.uint8), device=dev)
    o = torch.tensor(np.array(off, np.uint32).view(np.int32), device=dev)
    ln = torch.tensor(np.array([len(p) for p in payloads], np.uint32).view(np.int32), device=dev)
    sz = torch.tensor(np.array(sizes, np.uint32).view(np.int32), device=dev)
    cr = None if crcs is None else torch.tensor(np.array(crcs, np.uint32).view(np.int32), device=dev)
    dst = torch.zeros(max(1, n) * SLOT, dtype=torch.uint8, device=dev)
    st = torch.full((max(1, n),), -1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    N.check(N.lib().fc2_bgzf_inflate_launch(src.data_ptr(), o.data_ptr(), ln.data_ptr(), sz.data_ptr(),
                                            None if cr is None else cr.data_ptr(), dst.data_ptr(), st.data_ptr(), n,
                                            ctypes.c_void_p(stream)))
    torch.cuda.synchronize(dev)
    d = dst.cpu().numpy()
    return [d[i * SLOT:i * SLOT + sizes[i]].tobytes() for i in range(n)], st.cpu().numpy()[:n]


def _samples():
    rng = np.random.default_rng(1337)
    seqs = b"".join(open(os.path.join(GOLDEN, f), "rb").read() for f in ("test_ref.fa", "CDR1as_locus.fa"))
    acgt = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 70000)].tobytes()
    out = [b"", b"A", b"\x00" * 65536, b"AB" * 32768, bytes(rng.integers(0, 256, 65536, dtype=np.uint8)),
           acgt[:65280], (seqs * 30)[:65280], seqs[:1000], bytes(range(256)) * 200,
           b"".join(b"read%07d\tACGTNACGT\t" % i for i in range(3000))[:65536]]
    return out


@pytest.mark.parametrize("level", [0, 1, 6, 9])
@pytest.mark.parametrize("strategy", [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE,
                                      zlib.Z_FILTERED])
def test_inflate_equals_zlib(level, strategy):
    data = _samples()
    payloads = [_deflate(x, level, strategy) for x in data]
    got, st = _run(payloads, [len(x) for x in data])
    assert [int(x) for x in st] == [0] * len(data)
    assert got == data
    # the CRC-32 check on the device: the right ones pass, a wrong one is refused (status 16)
    crcs = [zlib.crc32(x) for x in data]
    _, st = _run(payloads, [len(x) for x in data], crcs)
    assert [int(x) for x in st] == [0] * len(data)
    _, st = _run(payloads, [len(x) for x in data], [c ^ (1 << (k % 32)) for k, c in enumerate(crcs)])
    assert [int(x) for x in st] == [16] * len(data)


def _bgzf_blocks(raw: bytes):
    """(payload, isize, crc) of every block of a BGZF file."""
    out, pos = [], 0
    while pos < len(raw):
        xlen = raw[pos + 10] | (raw[pos + 11] << 8)
        bsize = (raw[pos + 16] | (raw[pos + 17] << 8)) + 1
        payload = raw[pos + 12 + xlen:pos + bsize - 8]
        crc = int.from_bytes(raw[pos + bsize - 8:pos + bsize - 4], "little")
        isize = int.from_bytes(raw[pos + bsize - 4:pos + bsize], "little")
        out.append((payload, isize, crc))
        pos += bsize
    return out


def test_inflate_real_bam_blocks(tmp_path):
    """Every block of BAMs written by fc2_sam_to_bam (zlib level 1) and by the tests' BGZF writer
    (level 6, small blocks): the GPU output's CRC-32 equals the block's."""
    from samgen import bgzf_compress, sam_to_bam as py_sam_to_bam
    from test_native_caller import _rich_sam
    from find_circ2_amd.ingest import sam_to_bam
    sam = str(tmp_path / "rich.sam")
    _rich_sam(sam, 3000, seed=99)
    bam1 = str(tmp_path / "a.bam")
    sam_to_bam(sam, bam1)
    raw = str(tmp_path / "raw.bam")
    py_sam_to_bam(open(sam).read(), raw, compress="none")
    blocks = _bgzf_blocks(open(bam1, "rb").read()) + \
        _bgzf_blocks(bgzf_compress(open(raw, "rb").read(), block=3000, level=6))
    got, st = _run([b[0] for b in blocks], [b[1] for b in blocks], [b[2] for b in blocks])
    assert list(st) == [0] * len(blocks) and len(blocks) > 20
    assert [zlib.crc32(g) for g in got] == [b[2] for b in blocks]


def test_inflate_damaged_payloads_end_in_a_status():
    """Cut, bit-flipped, garbage and wrongly sized payloads: the launch completes, every block gets a
    status, and a block reported as inflated has the claimed size (its CRC-32 is the host's check)."""
    rng = np.random.default_rng(4711)
    data = _samples()
    good = [_deflate(x, lv) for x in data for lv in (1, 6)]
    sizes = [len(x) for x in data for _ in (1, 6)]
    payloads, want = [], []
    for p, n in zip(good, sizes):
        b = bytearray(p)
        kind = int(rng.integers(0, 5))
        if kind == 0 and len(b) > 4:
            b = b[:int(rng.integers(1, len(b)))]
        elif kind == 1 and len(b):
            for _ in range(8):
                k = int(rng.integers(0, len(b)))
                b[k] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:
            b = bytearray(rng.integers(0, 256, int(rng.integers(0, 4000)), dtype=np.uint8).tobytes())
        elif kind == 3:
            n = max(0, n - int(rng.integers(1, 100)))    # claimed size too small
        else:
            n = min(SLOT, n + int(rng.integers(1, 100)))  # claimed size too large
        payloads.append(bytes(b))
        want.append(n)
    payloads.append(_deflate(b"x" * 10))
    want.append(SLOT + 1)                               # over the BGZF limit
    got, st = _run(payloads, want)
    assert st[-1] != 0
    assert all(0 <= s <= 16 for s in st)
    for g, s, n in zip(got, st, want):
        if s == 0:
            assert len(g) == n


def _read_all(path, device=None, after=None):
    """Every handed-back fragment and the counts of a BAM read by the native ingest (GPU inflate on
    `device` -- from the start, or once `after` bytes were read -- or the CPU), and the inflate counts;
    or the error raised."""
    from find_circ2_amd.ingest import NativeIngest
    ing = None
    try:
        ing = NativeIngest(path, True)
        if device is not None and after is not None:
            ing.set_gpu_inflate_from(device, after)
        elif device is not None:
            ing.set_gpu_inflate(device)
        frags = []
        while not ing.eof:
            frags += [[(r.qname, r.flag, r.tid, r.pos, r.mapq, str(r.cigar), r.seq, r.qual, str(r.tags)) for r in f]
                      for f in ing.next_chunk(13, False, False, 97)]
        c = ing.counts
        return frags, tuple(getattr(c, f) for f, _ in c._fields_), ing.inflate_counts()
    except Exception as ex:          # noqa: BLE001 -- compared between the two paths
        return type(ex).__name__, str(ex), None
    finally:
        if ing is not None:
            ing.close()


def _bams(tmp_path):
    from samgen import bgzf_compress, sam_to_bam as py_sam_to_bam
    from test_native_caller import _rich_sam
    from find_circ2_amd.ingest import sam_to_bam
    sam = str(tmp_path / "rich.sam")
    _rich_sam(sam, 4000, seed=7)
    lvl1 = str(tmp_path / "lvl1.bam")
    sam_to_bam(sam, lvl1)                               # zlib level 1, 0xff00-byte blocks
    raw = str(tmp_path / "raw.bam")
    py_sam_to_bam(open(sam).read(), raw, compress="none")
    small = str(tmp_path / "small.bam")                 # level 6, 3000-byte blocks
    open(small, "wb").write(bgzf_compress(open(raw, "rb").read(), block=3000, level=6))
    tiny = str(tmp_path / "tiny.bam")                   # level 1, 700-byte blocks: GPU batches of chunks
    open(tiny, "wb").write(bgzf_compress(open(raw, "rb").read(), block=700, level=1))
    return lvl1, small, tiny


@pytest.mark.parametrize("batch", ["3", "64", "600"])
def test_ingest_gpu_inflate_equals_cpu(tmp_path, monkeypatch, batch):
    """The native ingest with its BGZF batches inflated on the GPU hands back the same fragments and
    counts as with the CPU inflate; every block after the batches read at the open went through the GPU."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("FC2_BGZF_BATCH", batch)
    for bam in _bams(tmp_path):
        cpu = _read_all(bam)
        gpu = _read_all(bam, 0)
        assert isinstance(cpu[0], list) and cpu[0], cpu
        assert cpu[:2] == gpu[:2]
        # the first two batches were under way before set_gpu_inflate (the open reads the header
        # from the first and starts the second)
        n_blocks = len(_bgzf_blocks(open(bam, "rb").read()))
        ahead = min(16, int(batch)) + int(batch)
        assert gpu[2] == (max(0, n_blocks - ahead), 0), (bam, gpu[2], n_blocks)
        assert cpu[2] == (0, 0)


def test_ingest_gpu_inflate_from_a_threshold(tmp_path, monkeypatch):
    """fc2_ingest_set_gpu_inflate_from (the CLI's default, 256 MiB): an input smaller than the threshold
    never touches the device (no block counted on it); one past it switches to the GPU mid-stream (the
    device's buffers made in the background from there) -- the same fragments and counts as the CPU
    inflate either way, at every batch size."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.delenv("FC2_GPU_INFLATE", raising=False)
    for batch in ("3", "64"):
        monkeypatch.setenv("FC2_BGZF_BATCH", batch)
        for bam in _bams(tmp_path):
            cpu = _read_all(bam)
            size = os.path.getsize(bam)
            never = _read_all(bam, 0, after=10 * size)
            assert never[:2] == cpu[:2] and never[2] == (0, 0), (bam, never[2])
            for after in (1, size // 3):
                mid = _read_all(bam, 0, after=after)
                assert mid[:2] == cpu[:2], (bam, after)
                n_blocks = len(_bgzf_blocks(open(bam, "rb").read()))
                assert sum(mid[2]) <= n_blocks, (bam, after, mid[2])


def test_ingest_gpu_inflate_corrupt_block_same_error(tmp_path, monkeypatch):
    """A damaged block: the same error with the GPU inflate as with the CPU's (the host's CRC check
    and CPU retry stand behind every GPU block)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("FC2_BGZF_BATCH", "4")
    _, small, _ = _bams(tmp_path)
    raw = bytearray(open(small, "rb").read())
    pos = 0
    for _ in range(9):                                   # the 10th block (the GPU's)
        pos += (raw[pos + 16] | (raw[pos + 17] << 8)) + 1
    for k in (40, 41, 300, 301):
        raw[pos + k] ^= 0x5A
    bad = str(tmp_path / "bad.bam")
    open(bad, "wb").write(bytes(raw))
    cpu, gpu = _read_all(bad), _read_all(bad, 0)
    assert cpu[2] is None and "corrupt BGZF block" in cpu[1], cpu
    assert gpu == cpu


def test_cli_bam_input_inflated_on_the_gpu(tmp_path, monkeypatch):
    """The CLI on a BAM reads it with the GPU inflate (run.log's process phases count the blocks) and
    writes the same files as with FC2_GPU_INFLATE=0; and with the buffers made in the background (the
    default) the same files again."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from test_cli import run_cli
    from test_cli_gpu import _compare, _sim_reads
    monkeypatch.setenv("FC2_BGZF_BATCH", "1")
    monkeypatch.setenv("FC2_GPU_INFLATE", "2")          # the device's buffers ready before the first read
    fa = os.path.join(GOLDEN, "CDR1as_locus.fa")
    rd = _sim_reads(fa, 3000, seed=5)
    rc1, o1 = run_cli(tmp_path, fa, rd, bam=True, evaluator=None, tag="gpu_inflate")
    monkeypatch.setenv("FC2_GPU_INFLATE", "0")
    rc2, o2 = run_cli(tmp_path, fa, rd, bam=True, evaluator=None, tag="cpu_inflate")
    assert rc1 == rc2 == 0
    _compare(o1, o2)

    def blocks(o):
        line = [l for l in open(os.path.join(o, "run.log")) if "process phases" in l][0]
        kv = dict(x.split("=") for x in line.split("process phases: ")[1].strip().split(", "))
        return float(kv["inflate_gpu_blocks"]), float(kv["inflate_cpu_blocks"])
    g1, c1 = blocks(o1)
    assert g1 >= 2 and c1 == 0
    assert blocks(o2) == (0.0, 0.0)
    monkeypatch.setenv("FC2_GPU_INFLATE", "1")
    rc3, o3 = run_cli(tmp_path, fa, rd, bam=True, evaluator=None, tag="gpu_inflate_background")
    assert rc3 == 0
    _compare(o1, o3)
    # the default: the GPU takes over past cli.GPU_INFLATE_AFTER bytes of input -- never for this
    # input; at a threshold of one byte, from the first batches whose device buffers are ready
    monkeypatch.delenv("FC2_GPU_INFLATE")
    rc4, o4 = run_cli(tmp_path, fa, rd, bam=True, evaluator=None, tag="gpu_inflate_default")
    assert rc4 == 0
    _compare(o1, o4)
    assert blocks(o4) == (0.0, 0.0)
    from find_circ2_amd import cli
    monkeypatch.setattr(cli, "GPU_INFLATE_AFTER", 1)
    rc5, o5 = run_cli(tmp_path, fa, rd, bam=True, evaluator=None, tag="gpu_inflate_default_low")
    assert rc5 == 0
    _compare(o1, o5)


def test_two_ingests_with_different_batches_share_the_pinned_pool(tmp_path, monkeypatch):
    """Two GPU-inflating ingests open at once with different batch sizes (so the pinned pool holds
    buffers of two sizes) read, interleaved, what each reads alone."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd.ingest import NativeIngest
    _, small, tiny = _bams(tmp_path)
    want = {}
    for bam, batch in ((small, "3"), (tiny, "600")):
        monkeypatch.setenv("FC2_BGZF_BATCH", batch)
        want[bam] = _read_all(bam)[:2]
    ings = []
    for bam, batch in ((small, "3"), (tiny, "600")):
        monkeypatch.setenv("FC2_BGZF_BATCH", batch)
        ing = NativeIngest(bam, True)
        ing.set_gpu_inflate(0)
        ings.append((bam, ing, []))
    try:
        while any(not ing.eof for _, ing, _ in ings):
            for _, ing, frags in ings:
                if not ing.eof:
                    frags += [[(r.qname, r.flag, r.tid, r.pos, r.mapq, str(r.cigar), r.seq, r.qual, str(r.tags))
                               for r in f] for f in ing.next_chunk(13, False, False, 31)]
        for bam, ing, frags in ings:
            c = ing.counts
            assert (frags, tuple(getattr(c, f) for f, _ in c._fields_)) == want[bam]
            assert ing.inflate_counts()[0] > 0 and ing.inflate_counts()[1] == 0
    finally:
        for _, ing, _ in ings:
            ing.close()
