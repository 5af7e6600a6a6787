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
