"""Every FC2_* environment knob of the read loop, at a value other than its default, writes the
default run's files byte for byte -- a knob may change speed, never an output (find_circ.py:1450-1486
grouping, :1276-1439 record_hits and :681-690 naming in input order, whatever the threads, blocks and
batches) -- and the knobs the library reads are exactly those INTEGRATION.md §4 lists and this file
runs.  The stress corner (one pinned parse block per chunk, blocks of one record, 16 workers on both
sides of the loop, a BGZF BAM whose fragments straddle blocks) is also run under ThreadSanitizer
(scripts/sanitize_host.sh tsan tests/test_knobs.py; profiles/r05/sanitize_tsan.txt)."""
import os
import re
import subprocess
import sys

import pytest

from test_ingest import same

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")

# knob -> a value other than the default (INTEGRATION.md §4 gives the defaults)
KNOBS = {
    "FC2_PARSE_THREADS": "1",
    "FC2_PARSE_INFLIGHT": "1",
    "FC2_PARSE_BLOCK": "1",          # the minimum: every record its own parse block
    "FC2_PIN_MAX": "1",
    "FC2_INGEST_THREADS": "1",
    "FC2_BGZF_BATCH": "1",
    "FC2_GPU_INFLATE": "1",          # (the CLI's GPU runs only; a no-op for the oracle runs here)
    "FC2_NEXT_THREADS": "16",
    "FC2_CALLER_THREADS": "16",
    "FC2_CALLER_MIN_RANGE": "1",
    "FC2_LIBDEFLATE": "0",           # zlib instead of libdeflate (read once per process)
    "FC2_CALLER_TIMING": "1",        # diagnostics on stderr (read once per process)
}

STRESS = dict(FC2_PIN_MAX="1", FC2_PARSE_BLOCK="1", FC2_PARSE_INFLIGHT="2", FC2_NEXT_THREADS="16",
              FC2_CALLER_THREADS="16", FC2_CALLER_MIN_RANGE="1", FC2_BGZF_BATCH="1", FC2_INGEST_THREADS="4")


def _library_knobs():
    names = set()
    d = os.path.join(ROOT, "find_circ2_amd", "csrc")
    for f in os.listdir(d):
        if f.endswith((".cpp", ".h", ".hip")):
            names |= set(re.findall(r'getenv\("(FC2_[A-Z0-9_]+)"\)', open(os.path.join(d, f)).read()))
    return names


def test_knob_inventory():
    """The library reads the knobs INTEGRATION.md lists, and each is run below."""
    listed = set(re.findall(r"^\| `(FC2_[A-Z0-9_]+)", open(os.path.join(ROOT, "INTEGRATION.md")).read(), re.M))
    assert _library_knobs() == set(KNOBS) == listed, (_library_knobs() ^ set(KNOBS), listed ^ set(KNOBS))


@pytest.fixture(scope="module")
def bam_input(tmp_path_factory):
    """The rich bwa-mem-shaped input (test_native_caller._rich_sam) as a BGZF BAM of 3 kB blocks, so
    fragments straddle BGZF blocks, inflate batches and parse blocks."""
    from samgen import bgzf_compress, sam_to_bam
    from test_native_caller import _rich_sam
    d = tmp_path_factory.mktemp("knobs")
    sam = str(d / "rich.sam")
    fa = _rich_sam(sam, 700, seed=3131)
    raw = str(d / "raw.bam")
    sam_to_bam(open(sam).read(), raw, compress="none")
    bam = str(d / "rich.bam")
    open(bam, "wb").write(bgzf_compress(open(raw, "rb").read(), block=3000, level=1))
    return fa, sam, bam


def _run(fa, inp, out, env=None, extra=()):
    e = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, TESTS]))
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(TESTS, "cli_oracle_main.py"), "-G", fa, "-o", out, "-n", "k",
                        "-q", "--chunk-size", "53"] + list(extra) + [inp], env=e, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    return r


@pytest.fixture(scope="module")
def default_out(bam_input, tmp_path_factory):
    fa, sam, bam = bam_input
    o = str(tmp_path_factory.mktemp("default") / "o")
    _run(fa, bam, o)
    return o


@pytest.mark.parametrize("knob", sorted(KNOBS))
def test_knob_changes_no_byte(bam_input, default_out, tmp_path, knob):
    fa, sam, bam = bam_input
    o = str(tmp_path / "o")
    r = _run(fa, bam, o, {knob: KNOBS[knob]})
    same(default_out, o)
    if knob == "FC2_CALLER_TIMING":
        assert b"submit nf=" in r.stderr


@pytest.mark.parametrize("extra", [[], ["--all-hits", "--non-canonical"]])
def test_stress_corner_equals_python_loop(bam_input, tmp_path, extra):
    """Every sizing knob at its most fragmenting setting at once against the Python read loop (the
    pinned-batch lifetimes and records read in place across parse blocks, on 16 + 16 workers)."""
    from find_circ2_amd import cli
    from oracle_engine import oracle_evaluator_factory
    fa, sam, bam = bam_input
    o1 = str(tmp_path / "py")
    assert cli.main(["-G", fa, "-o", o1, "-n", "k", "-q", "--python-caller", "--chunk-size", "53"] + extra + [sam],
                    evaluator_factory=oracle_evaluator_factory) == 0
    o2 = str(tmp_path / "stress")
    _run(fa, bam, o2, STRESS, extra)
    same(o1, o2)


def test_threads_option_sizes_the_pools(bam_input, default_out, tmp_path):
    """--threads N (cliopts.apply_threads) sizes every native pool through the knobs above: the recording
    side's phase A runs on at most N ranges, and the files are the default run's."""
    fa, sam, bam = bam_input
    o = str(tmp_path / "o")
    r = _run(fa, bam, o, {"FC2_CALLER_TIMING": "1"}, extra=["--threads", "3"])
    same(default_out, o)
    ts = [int(x) for x in re.findall(rb"submit nf=\d+ T=(\d+)", r.stderr)]
    assert ts and max(ts) <= 3
