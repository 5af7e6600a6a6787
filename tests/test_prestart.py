"""prestart.py: ``python -m find_circ2_amd.cli`` opens the FASTA and builds the device contexts on a
thread before the package imports numpy; main adopts them.  Without a GPU (CPU suite) the adopted
path must fail exactly as main's own did (the device error in run.log, status 1), a FASTA the
reference's index() rejects must raise the same error, -G <folder> must go to the reference's dummy
mode with its warning (find_circ.py:338-345), and --help / --version / bad arguments must behave as
without it.  On a GPU the -m CLI equals the oracle CLI, also in dummy mode and with --gpus 2."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import GOLDEN, ROOT
from find_circ2_amd import cli, prestart
from samgen import sam_text
from bwa_emul import read_fasta
from test_cli import _reads, run_cli


def _gpu():
    try:
        from find_circ2_amd.ctxpipe import device_count
        return device_count() > 0
    except Exception:
        return False


def _m(args, **kw):
    return subprocess.run([sys.executable, "-m", "find_circ2_amd.cli"] + list(args), cwd=ROOT,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300, **kw)


def _inproc(args):
    code = "import sys; from find_circ2_amd import cli; sys.exit(cli.main(%r))" % (list(args),)
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                          timeout=300)


def _sam(tmp_path, fa):
    p = str(tmp_path / "in.sam")
    open(p, "w").write(sam_text(read_fasta(fa), _reads(os.path.join(GOLDEN, "test_reads.fa"))))
    return p


def test_help_version_and_bad_arguments_unchanged():
    for args in (["--version"], ["--help"], ["--no-such-flag"], ["-a", "x"]):
        a, b = _m(args), _inproc(args)
        assert a.returncode == b.returncode, args
        assert a.stdout.replace(b"-m", b"") == b.stdout.replace(b"-c", b"") or args == ["--help"], args
        if args == ["--help"]:
            assert a.stdout.count(b"--genome") == 1


def test_start_skips_what_main_does_alone(capsys):
    saved = prestart._started
    try:
        for argv in (["--help"], ["--version"], ["-x"], [], ["-G", "g.fa", "--python-caller"],
                     ["-G", "g.fa", "--python-ingest"], ["-S", "hs", "-G", "g.fa"], ["-G", "g.fa", "--device", "cuda:x"]):
            prestart._started = None
            prestart.start(argv)
            assert prestart._started is None, argv
        out = capsys.readouterr()
        assert out.out == "" and out.err == ""
    finally:
        prestart._started = saved


def test_take_discards_a_prestart_for_other_options(tmp_path):
    fa = str(tmp_path / "g.fa")
    shutil.copy(os.path.join(GOLDEN, "test_ref.fa"), fa)
    p = prestart.Prestart(fa, "cuda:0", 1)
    saved = prestart._started
    try:
        prestart._started = p
        opts, _ = cli.build_parser().parse_args(["-G", fa, "--gpus", "2"])
        assert prestart.take(opts) is None and prestart._started is None
        assert p.fasta is None and p.ctxs == []
        p2 = prestart.Prestart(fa, "cuda:0", 1)
        prestart._started = p2
        opts, _ = cli.build_parser().parse_args(["-G", fa])
        assert prestart.take(opts) is p2 and prestart.take(opts) is None
        p2.thread.join()
        p2.discard()
    finally:
        prestart._started = saved


@pytest.mark.skipif(_gpu(), reason="a GPU is present")
def test_no_gpu_fails_as_main_does(tmp_path):
    fa = str(tmp_path / "g.fa")
    shutil.copy(os.path.join(GOLDEN, "test_ref.fa"), fa)
    sam = _sam(tmp_path, fa)
    a = _m(["-G", fa, "-o", str(tmp_path / "m"), "-q", sam])
    b = _inproc(["-G", fa, "-o", str(tmp_path / "c"), "-q", sam])
    assert a.returncode == b.returncode == 1
    la, lb = (open(str(tmp_path / o / "run.log")).read() for o in ("m", "c"))
    assert "fc2_ctx_create" in la and "fc2_ctx_create" in lb
    err = [l for l in la.splitlines() if "libfc2 error" in l]
    assert err and err[-1].split("\t")[-1] in lb


@pytest.mark.skipif(_gpu(), reason="a GPU is present")
def test_no_gpu_dummy_mode_warns_then_fails(tmp_path):
    folder = tmp_path / "folder"
    folder.mkdir()
    shutil.copy(os.path.join(GOLDEN, "test_ref.fa"), str(folder / "x.fa"))
    sam = _sam(tmp_path, os.path.join(GOLDEN, "test_ref.fa"))
    a = _m(["-G", str(folder), "-o", str(tmp_path / "m"), "-q", sam])
    assert a.returncode == 1
    log = open(str(tmp_path / "m" / "run.log")).read()
    assert "Switching to dummy mode" in log and "fc2_ctx_create" in log


def test_fasta_format_error_raises_as_main_does(tmp_path):
    fa = str(tmp_path / "bad.fa")
    open(fa, "w").write(">\nACGT\n")                    # an empty header: index() raises IndexError
    sam = str(tmp_path / "in.sam")
    open(sam, "w").write("@SQ\tSN:b\tLN:4\n")
    a = _m(["-G", fa, "-o", str(tmp_path / "m"), "-q", sam])
    b = _inproc(["-G", fa, "-o", str(tmp_path / "c"), "-q", sam])
    assert a.returncode == b.returncode == 1
    last = lambda r: [l for l in r.stderr.decode().splitlines() if l.strip()][-1]      # noqa: E731
    assert last(a) == last(b) and "libfc2 error -3" in last(a), last(a)


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--gpus", "2", "--all-hits"]])
@pytest.mark.parametrize("folder", [False, True], ids=["fasta", "folder"])
def test_gpu_m_cli_equals_oracle_cli(tmp_path, extra, folder):
    if not _gpu():
        pytest.skip("no GPU")
    from test_cli_gpu import _compare
    fa = os.path.join(GOLDEN, "CDR1as_locus.fa")
    g = str(tmp_path / "g.fa")
    shutil.copy(fa, g)
    if folder:
        os.makedirs(str(tmp_path / "folder"))
        shutil.copy(fa, str(tmp_path / "folder" / "x.fa"))
        g = str(tmp_path / "folder")
    rd = _reads(os.path.join(GOLDEN, "cdr1as_reads.fa"))
    rc1, o1 = run_cli(tmp_path, fa, rd, extra=[e for e in extra if e not in ("--gpus", "2")], tag="oracle",
                      genome_arg=g)
    sam = str(tmp_path / "in.sam")              # (run_cli wrote it)
    r = _m(["-G", g, "-o", str(tmp_path / "m"), "-n", "test", "-q"] + extra + [sam])
    assert rc1 == 0 and r.returncode == 0, r.stderr.decode()[-2000:]
    _compare(o1, str(tmp_path / "m"))
    log = open(str(tmp_path / "m" / "run.log")).read()
    assert ("Switching to dummy mode" in log) == folder
    assert "process phases" in log and "torch_loaded=0" in log
    if not extra:                               # the default loop never imports numpy (_lazy.py)
        assert "numpy_loaded=0" in log


def test_package_names_and_submodules_resolve_lazily():
    """find_circ2_amd imports its names on first use (PEP 562): every exported name and every submodule
    reached as an attribute (``find_circ2_amd._native``, as __graft_entry__.build does) resolves, in a
    fresh interpreter where nothing was imported before; an unknown name raises AttributeError."""
    code = ("import find_circ2_amd as f, sys\n"
            "assert 'numpy' not in sys.modules\n"
            "assert f._native.FC2_OK == 0 and f.hotpath.Options is f.Options and f.ctxpipe.CtxPipeline\n"
            "for n in f.__all__: getattr(f, n)\n"
            "try:\n    f.no_such_name\nexcept AttributeError:\n    pass\nelse:\n    raise SystemExit(1)\n"
            "import __graft_entry__ as g\n"
            "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == b"ok", r.stderr.decode()[-2000:]
