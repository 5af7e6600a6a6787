"""The CLI with the GPU evaluator produces byte-identical output files to the CLI
with the CPU oracle evaluator (same host logic, different breakpoint search)."""
import gzip
import os

import pytest

from conftest import GOLDEN
from synth_small import load_genome, make_spans
from test_cli import _reads, run_cli

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

FILES = ("circ_splice_sites.bed", "lin_splice_sites.bed", "multi_events.tsv", "test_results.tsv")


def _compare(o1, o2):
    for f in FILES:
        p1, p2 = os.path.join(o1, f), os.path.join(o2, f)
        if os.path.exists(p1) or os.path.exists(p2):
            assert open(p1).read() == open(p2).read(), f
    with gzip.open(os.path.join(o1, "spliced_reads.fastq.gz"), "rt") as a, \
            gzip.open(os.path.join(o2, "spliced_reads.fastq.gz"), "rt") as b:
        assert a.read() == b.read()


def _sim_reads(fa, n, seed):
    g = load_genome(fa)
    spans = make_spans(g, n, seed=seed, L=(60, 150), p_readN=0.02, p_lower=0.0, p_clip=0.0, mut=0.005)
    return [("sim%05d" % i, s.read_part.decode().upper()) for i, s in enumerate(spans)]


@pytest.mark.parametrize("fa,reads", [("test_ref.fa", "test_reads.fa"), ("CDR1as_locus.fa", "cdr1as_reads.fa")])
@pytest.mark.parametrize("extra", [[], ["--non-canonical", "--all-hits"], ["--strand-pref", "-d", "0"]])
def test_gpu_cli_equals_oracle_cli_golden(tmp_path, fa, reads, extra):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fa = os.path.join(GOLDEN, fa)
    rd = _reads(os.path.join(GOLDEN, reads))
    rc1, o1 = run_cli(tmp_path, fa, rd, extra=["--test"] + extra, tag="oracle")
    rc2, o2 = run_cli(tmp_path, fa, rd, extra=["--test"] + extra, evaluator=None, tag="gpu")
    assert rc1 == rc2 == 0
    _compare(o1, o2)


@pytest.mark.parametrize("fa", ["CDR1as_locus.fa", "test_ref.fa"])
def test_gpu_cli_equals_oracle_cli_simulated(tmp_path, fa):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fa = os.path.join(GOLDEN, fa)
    rd = _sim_reads(fa, 1500, seed=11358)
    for extra in ([], ["--non-canonical", "--all-hits", "--chunk-size", "97"]):
        rc1, o1 = run_cli(tmp_path, fa, rd, extra=extra, tag="oracle")
        rc2, o2 = run_cli(tmp_path, fa, rd, extra=extra, evaluator=None, tag="gpu")
        assert rc1 == rc2
        if rc1 == 0:
            _compare(o1, o2)


@pytest.mark.parametrize("extra", [[], ["--all-hits", "--non-canonical", "--strand-pref"], ["-d", "0"]])
def test_gpu_native_caller_equals_oracle_python_caller(tmp_path, extra):
    """The shipped configuration (C++ read loop + HIP scan) against the Python read loop
    with the CPU oracle, on the rich mixed input of test_native_caller.py."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    from test_ingest import same
    from test_native_caller import _rich_sam
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 2500, seed=97)
    o1, o2 = str(tmp_path / "oracle_py"), str(tmp_path / "gpu_native")
    rc1 = cli.main(["-G", fa, "-o", o1, "-n", "mix", "-q", "--python-caller"] + extra + [sam],
                   evaluator_factory=oracle_evaluator_factory)
    rc2 = cli.main(["-G", fa, "-o", o2, "-n", "mix", "-q"] + extra + [sam])
    assert rc1 == rc2 == 0
    same(o1, o2)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_gpu_native_caller_on_mutated_input(tmp_path, seed):
    """Fuzzed records (tests/test_caller_fuzz.py: N / IUPAC / lower-case read bytes, CIGAR
    variants, flag bits, AS/XS changes) through the shipped CLI vs the Python loop + oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    from test_caller_fuzz import _mutate
    from test_ingest import same
    from test_native_caller import _rich_sam
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, 600, seed=700 + seed)
    lines = open(sam0).read().splitlines()
    rng = np.random.default_rng(seed)
    body = _mutate([l for l in lines if not l.startswith("@")], rng, rate=0.03, fatal=False)
    sam = str(tmp_path / "m.sam")
    open(sam, "w").write("\n".join([l for l in lines if l.startswith("@")] + body) + "\n")
    extra = [[], ["--all-hits", "--non-canonical"]][seed % 2]
    o1, o2 = str(tmp_path / "oracle_py"), str(tmp_path / "gpu_native")
    rc1 = cli.main(["-G", fa, "-o", o1, "-q", "--python-caller"] + extra + [sam],
                   evaluator_factory=oracle_evaluator_factory)
    rc2 = cli.main(["-G", fa, "-o", o2, "-q"] + extra + [sam])
    assert rc1 == rc2 == 0
    same(o1, o2)


@pytest.mark.parametrize("extra", [[], ["--all-hits", "--non-canonical", "--chunk-size", "37"],
                                   ["--chunk-size", "11", "-d", "0"]])
def test_gpu_cli_two_gpus_equals_one(tmp_path, extra):
    """--gpus 2 (chunks dealt round-robin to two scanners -- two devices, or two streams sharing
    cuda:0 on a one-GPU box -- results merged in input order) writes the files --gpus 1 writes,
    byte for byte, and both equal the Python loop with the CPU oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    from test_ingest import same
    from test_native_caller import _rich_sam
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 2500, seed=1234)
    outs = {}
    for tag, more in (("g1", ["--gpus", "1"]), ("g2", ["--gpus", "2"]), ("g3", ["--gpus", "3"])):
        o = str(tmp_path / tag)
        assert cli.main(["-G", fa, "-o", o, "-n", "mix", "-q"] + extra + more + [sam]) == 0
        outs[tag] = o
    o = str(tmp_path / "oracle_py")
    assert cli.main(["-G", fa, "-o", o, "-n", "mix", "-q", "--python-caller"] + extra + [sam],
                    evaluator_factory=oracle_evaluator_factory) == 0
    same(outs["g1"], outs["g2"])
    same(outs["g1"], outs["g3"])
    same(o, outs["g2"])


@pytest.mark.parametrize("gpus", ["9", "20"])
def test_gpu_cli_many_gpu_entries_read_ahead_within_the_queue_limit(tmp_path, gpus):
    """--gpus 9 / 20 on a one-GPU box (entries wrap round the devices present: 9 or 20 scanners): the
    read-ahead depth stays within the chunks fc2_caller_next keeps queued (FC2_CALLER_MAX_QUEUED), so
    tiny chunks read ahead while the genome loads do not stop the run, and the files equal
    --gpus 1's."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import cli
    from test_ingest import same
    from test_native_caller import _rich_sam
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 3000, seed=4321)
    o1, o2 = str(tmp_path / "g1"), str(tmp_path / ("g" + gpus))
    assert cli.main(["-G", fa, "-o", o1, "-q", "--chunk-size", "5", "--gpus", "1", sam]) == 0
    assert cli.main(["-G", fa, "-o", o2, "-q", "--chunk-size", "5", "--gpus", gpus, sam]) == 0
    same(o1, o2)


def test_gpu_pipeline_readahead_many_chunks(tmp_path):
    """ScanPipeline through the native loop with tiny chunks (hundreds of chunks, two in flight
    per scanner, staging slots reused) on the golden reads: the same files as the oracle CLI."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fa = os.path.join(GOLDEN, "CDR1as_locus.fa")
    rd = _sim_reads(fa, 1200, seed=5)
    for extra in (["--chunk-size", "3"], ["--chunk-size", "5", "--gpus", "2", "--all-hits", "--non-canonical"]):
        rc1, o1 = run_cli(tmp_path, fa, rd, extra=[e for e in extra if e not in ("--gpus", "2")], tag="oracle")
        rc2, o2 = run_cli(tmp_path, fa, rd, extra=extra, evaluator=None, tag="gpu")
        assert rc1 == rc2
        if rc1 == 0:
            _compare(o1, o2)


@pytest.mark.parametrize("gpus", ["1", "2"])
def test_gpu_bam_out_equals_oracle(tmp_path, gpus):
    """-B (the sequential loop: the BAM writer needs each chunk's verdicts before the next chunk's
    records are written) through the HIP scan, on one or two scanners: the same
    spliced_alignments.bam records and the same text files as the oracle run."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    from test_bam_out import read_bam
    from test_ingest import same
    from test_native_caller import _rich_sam
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 1500, seed=31)
    o1, o2 = str(tmp_path / "oracle"), str(tmp_path / "gpu")
    common = ["-G", fa, "-q", "-B", "--chunk-size", "13"]
    assert cli.main(common + ["-o", o1, sam], evaluator_factory=oracle_evaluator_factory) == 0
    assert cli.main(common + ["-o", o2, "--gpus", gpus, sam]) == 0
    same(o1, o2)
    b1 = read_bam(os.path.join(o1, "spliced_alignments.bam"))
    b2 = read_bam(os.path.join(o2, "spliced_alignments.bam"))
    assert len(b1[2]) > 1000 and b1 == b2


def test_gpu_cli_multi_block_sam(tmp_path):
    """A 9 MiB SAM (several 4 MiB blocks for the splitter and the two parser threads) through the
    shipped CLI with the HIP scan on two scanners: the same files as the Python loop + oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    from test_ingest import same
    from test_native_caller import _large_sam
    fa, hdr, body = _large_sam(tmp_path, 20000, seed=31415)
    sam = str(tmp_path / "big.sam")
    open(sam, "w").write("\n".join(hdr + body) + "\n")
    assert os.path.getsize(sam) > (9 << 20)
    o1, o2 = str(tmp_path / "oracle_py"), str(tmp_path / "gpu")
    assert cli.main(["-G", fa, "-o", o1, "-q", "--python-caller", sam], evaluator_factory=oracle_evaluator_factory) == 0
    assert cli.main(["-G", fa, "-o", o2, "-q", "--gpus", "2", sam]) == 0
    same(o1, o2)


@pytest.mark.parametrize("extra", [[], ["--all-hits", "--non-canonical", "--gpus", "2"]])
def test_gpu_cli_bam_on_stdin_equals_oracle_cli(tmp_path, extra):
    """north_star's form: ``samtools view -b ... | python -m find_circ2_amd.cli -G g.fa -o out`` -- a
    BGZF BAM piped into the shipped CLI (its own process, HIP scan) writes the files the Python loop
    with the CPU oracle writes from the SAM by path (find_circ.py:467-469: stdin read by what it is)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import subprocess
    import sys
    from conftest import ROOT
    from find_circ2_amd import cli
    from find_circ2_amd.ingest import sam_to_bam
    from oracle_engine import oracle_evaluator_factory
    from test_ingest import same
    from test_native_caller import _large_sam
    fa, hdr, body = _large_sam(tmp_path, 8000, seed=2718)
    sam = str(tmp_path / "in.sam")
    open(sam, "w").write("\n".join(hdr + body) + "\n")
    bam = str(tmp_path / "in.bam")
    sam_to_bam(sam, bam)
    o1, o2 = str(tmp_path / "oracle_py"), str(tmp_path / "gpu_stdin")
    assert cli.main(["-G", fa, "-o", o1, "-q", "--python-caller"] + [e for e in extra if e not in ("--gpus", "2")]
                    + [sam], evaluator_factory=oracle_evaluator_factory) == 0
    feeder = subprocess.Popen(["cat", bam], stdout=subprocess.PIPE)
    r = subprocess.run([sys.executable, "-m", "find_circ2_amd.cli", "-G", fa, "-o", o2, "-q"] + extra, cwd=ROOT,
                       stdin=feeder.stdout, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    feeder.stdout.close()
    feeder.wait()
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    same(o1, o2)


@pytest.mark.parametrize("extra", [[], ["--python-caller"], ["--non-canonical", "--all-hits", "-d", "0"]])
def test_gpu_cli_genome_folder_dummy_mode_equals_oracle(tmp_path, extra):
    """-G <folder> (find_circ.py:386): file() raises IOError (:117, :124), GenomeAccessor runs in
    all-N dummy mode (:338-345) -- the GPU CLI writes what the oracle CLI writes, no junctions."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import shutil
    fa = os.path.join(GOLDEN, "CDR1as_locus.fa")
    folder = tmp_path / "folder"
    folder.mkdir()
    shutil.copy(fa, str(folder / "chr_CDR1as.fa"))
    rd = _reads(os.path.join(GOLDEN, "cdr1as_reads.fa"))
    rc1, o1 = run_cli(tmp_path, fa, rd, extra=extra, tag="oracle", genome_arg=str(folder))
    rc2, o2 = run_cli(tmp_path, fa, rd, extra=extra, evaluator=None, tag="gpu", genome_arg=str(folder))
    assert rc1 == rc2 == 0
    _compare(o1, o2)
    for o in (o1, o2):
        assert "Switching to dummy mode" in open(os.path.join(o, "run.log")).read()
        assert [l for l in open(os.path.join(o, "circ_splice_sites.bed")) if not l.startswith("#")] == []


@pytest.mark.parametrize("opts", [["-a", "2", "-m", "2", "-d", "0"], ["-a", "10", "-m", "12", "-d", "0"],
                                  ["-a", "2", "-m", "2", "-d", "2"], ["-a", "3", "-m", "3", "-d", "1",
                                                                      "--non-canonical"]])
def test_gpu_cli_asize_le_margin_equals_oracle(tmp_path, opts):
    """asize <= margin (find_circ.py:882, :895): with -d 0 every span finds no breakpoint and the
    run completes; with -d > 0 numpy's shape failure (:861-863) ends the run (exit 1) at the first
    span record_hits evaluates -- the GPU CLI does what the oracle CLI does."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fa = os.path.join(GOLDEN, "test_ref.fa")
    rd = _reads(os.path.join(GOLDEN, "test_reads.fa"))
    for extra in (opts, opts + ["--python-caller"]):
        rc1, o1 = run_cli(tmp_path, fa, rd, extra=extra, tag="oracle")
        rc2, o2 = run_cli(tmp_path, fa, rd, extra=extra, evaluator=None, tag="gpu")
        assert rc1 == rc2
        if "-d" in opts and opts[opts.index("-d") + 1] == "0":
            assert rc1 == 0
        if rc1 == 0:
            _compare(o1, o2)


@pytest.mark.parametrize("extra", [[], ["--python-caller"]])
def test_gpu_cli_none_aend_span_raises_where_oracle_does(tmp_path, extra):
    """A spliced read whose supplementary record -- the B segment, after a primary aligned from
    query position 0 -- has CIGAR '*' (align_B.aend None): the GPU runs (native loop, and the Python
    loop with the GPU evaluator) fail at that fragment with the reference's TypeError of
    `B.aend - eff_a` (find_circ.py:902), after recording the fragments before it -- the same
    partial files as the oracle CLI."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import re
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    from test_native_caller import _rich_sam
    sam = str(tmp_path / "rich.sam")
    fa = _rich_sam(sam, 700, seed=77)
    lines = open(sam).read().splitlines()
    recs = [l.split("\t") for l in lines if not l.startswith("@")]
    supp = {f[0] for f in recs if int(f[1]) & 2048}
    cands = [f[0] for f in recs if f[0] in supp and not int(f[1]) & 2048 and re.match(r"^\d+M\d+S$", f[5])]
    msg = "unsupported operand type(s) for -: 'NoneType' and 'int'"
    for target in cands[len(cands) // 2:][:6]:
        out = []
        for l in lines:
            f = l.split("\t")
            if not l.startswith("@") and f[0] == target and int(f[1]) & 2048:
                f[5] = "*"
                if f[9] == "*":
                    f[9], f[10] = "A" * 60, "I" * 60
            out.append("\t".join(f))
        p = str(tmp_path / "bad.sam")
        open(p, "w").write("\n".join(out) + "\n")
        o1, o2 = str(tmp_path / ("oracle_" + target)), str(tmp_path / ("gpu_" + target))
        rc1 = cli.main(["-G", fa, "-o", o1, "-q", "--python-caller", p], evaluator_factory=oracle_evaluator_factory)
        if rc1 != 1 or msg not in open(os.path.join(o1, "run.log")).read():
            continue                             # the span is not evaluated (not unique enough)
        rc2 = cli.main(["-G", fa, "-o", o2, "-q"] + extra + [p])
        assert rc2 == 1
        err = [l for l in open(os.path.join(o2, "run.log")) if "Error" in l]
        assert err and msg in err[-1], err
        _compare(o1, o2)
        return
    pytest.fail("no fragment whose B segment's span is evaluated")


@pytest.mark.parametrize("extra", [[], ["--all-hits", "--non-canonical", "-d", "3"], ["--gpus", "2"]],
                         ids=["default", "all-hits", "gpus2"])
@pytest.mark.parametrize("mode", [[], ["--python-caller"]], ids=["native", "python-caller"])
def test_gpu_cli_long_reads_equal_oracle(tmp_path, extra, mode):
    """Read parts over FC2_MAX_READ_LEN (33-36 kb) go through the GPU long path (fc2_bp_scan_long_launch;
    the reference's x-loop has no length limit, find_circ.py:873, :904-906): the GPU CLI, native or
    Python read loop, writes the files of the Python loop with the CPU oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    from test_ingest import same
    from test_read_limits import _long_read_genome, _long_reads, _sam_of
    L = 36000
    g = _long_read_genome(L)
    reads = _long_reads(g, L)
    fa = str(tmp_path / "g.fa")
    with open(fa, "w") as f:
        for c, sq in g.items():
            t = sq.decode()
            f.write(">%s\n" % c + "".join(t[i:i + 60] + "\n" for i in range(0, len(t), 60)))
    sam = str(tmp_path / "in.sam")
    open(sam, "w").write(_sam_of(g, reads))
    o1, o2 = str(tmp_path / "oracle_py"), str(tmp_path / "gpu")
    rc1 = cli.main(["-G", fa, "-o", o1, "-n", "lr", "-q", "--python-caller"] + [e for e in extra if e != "--gpus"
                   and e != "2"] + [sam], evaluator_factory=oracle_evaluator_factory)
    rc2 = cli.main(["-G", fa, "-o", o2, "-n", "lr", "-q"] + mode + extra + [sam])
    assert rc1 == rc2 == 0
    same(o1, o2)
    assert "g2\t2000\t%d\t" % (2000 + (L - 2000) + 8000) in open(os.path.join(o2, "circ_splice_sites.bed")).read()


def test_gpu_cli_float_as_xs_equals_oracle(tmp_path):
    """Float AS / XS tags through the GPU CLI: the native loop's Python-2 arithmetic and formatting of
    best_qual_left/right (find_circ.py:556-566, :593) equal the Python loop with the CPU oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    from test_ingest import same
    from test_native_caller import _float_tags, _retag, _rich_sam
    sam0 = str(tmp_path / "base.sam")
    fa = _rich_sam(sam0, 800, seed=5150)
    sam = str(tmp_path / "float.sam")
    open(sam, "w").write("\n".join(_retag(open(sam0).read().splitlines(), np.random.default_rng(77), _float_tags))
                         + "\n")
    o1, o2 = str(tmp_path / "oracle_py"), str(tmp_path / "gpu")
    rc1 = cli.main(["-G", fa, "-o", o1, "-n", "mix", "-q", "--python-caller", sam],
                   evaluator_factory=oracle_evaluator_factory)
    rc2 = cli.main(["-G", fa, "-o", o2, "-n", "mix", "-q", sam])
    assert rc1 == rc2 == 0
    same(o1, o2)


def test_gpu_cli_empty_bam_named_input_fails(tmp_path):
    """An empty x.bam (a crashed aligner's leftover): pysam's header check raises ValueError where
    the reference opens it (find_circ.py:463-466) -- the GPU CLI exits 1 with that error."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from find_circ2_amd import cli
    p = str(tmp_path / "x.bam")
    open(p, "wb").close()
    o = str(tmp_path / "o")
    assert cli.main(["-G", os.path.join(GOLDEN, "test_ref.fa"), "-o", o, "-q", p]) == 1
    assert "ValueError: file has no sequences defined (mode='rb')" in open(os.path.join(o, "run.log")).read()
