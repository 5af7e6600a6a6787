"""BASELINE configs[0]: the reference's regression targets (test_data/Makefile: unit_test, cdr1as_test
and hek_test2's re-run procedure) through scripts/test_data_targets.py -- on CPU with the oracle as
the search (plumbing, as configs[0] is), and on the GPU with the shipped HIP scan.  The HEK293 data
and hg19 are absent (.MISSING_LARGE_BLOBS), so hek_test2's procedure runs on the golden genomes."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _target(name, tmp_path, gpu=False):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "test_data_targets.py"), name, "--out",
                        str(tmp_path)] + (["--gpu"] if gpu else []), cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    return r.stdout + r.stderr


@pytest.mark.parametrize("name", ["unit_test", "cdr1as_test", "rerun_test"])
def test_target_cpu(name, tmp_path):
    out = _target(name, tmp_path)
    if name != "unit_test":
        assert "files contain identical splice sites!" in out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["unit_test", "cdr1as_test", "rerun_test"])
def test_target_gpu(name, tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = _target(name, tmp_path, gpu=True)
    if name != "unit_test":
        assert "files contain identical splice sites!" in out
