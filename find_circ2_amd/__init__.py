"""find_circ2_amd -- MI355X-native breakpoint search for find_circ2.

One hot path of find_circ2 (find_circ.py 1.99), ``JunctionSpan.find_breakpoints``
plus its genome window fetch, as hand-written HIP kernels for gfx950 behind a
C ABI (include/fc2_bp.h, libfc2.so).  See DESIGN.md.
"""
import os as _os
import sys as _sys

# `python -m find_circ2_amd.<module>` (the CLI): nothing of this package calls BLAS, and OpenBLAS's
# thread pool, started when numpy is first imported (one thread per OMP_NUM_THREADS), costs the
# process ~0.1 s of start-up.  While -m locates the module, sys.argv[0] is "-m"; an explicit
# OPENBLAS_NUM_THREADS stays as given, and a library import leaves the environment alone.
if _sys.argv[:1] == ["-m"] and "numpy" not in _sys.modules:
    _os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
# `python -m find_circ2_amd.cli`: the device genome is started now, before the imports below (prestart.py)
_orig = getattr(_sys, "orig_argv", [])
if _sys.argv[:1] == ["-m"] and "-m" in _orig and _orig[_orig.index("-m") + 1:][:1] == ["find_circ2_amd.cli"]:
    from . import prestart as _prestart
    _prestart.start(_sys.argv[1:])

# the package's names are imported on first use (PEP 562): `python -m find_circ2_amd.cli` then loads
# only what the CLI needs -- neither numpy nor torch for the default loop
_EXPORTS = {"Genome": "genome", "sq_table": "genome", "synthetic_n_intervals": "genome",
            **{k: "hotpath" for k in ("BreakpointEngine", "BreakpointError", "CompactResults", "JunctionSpan",
                                      "Options", "PairBatch", "ScanOutput", "Splice", "SynthConfig", "compact",
                                      "decode_splices", "expand", "first_tie_arrays", "gtag_str", "reorder", "scan",
                                      "splices_or_raise")}}


def __getattr__(name):
    import importlib
    mod = _EXPORTS.get(name)
    if mod is not None:
        value = getattr(importlib.import_module("." + mod, __name__), name)
    elif not name.startswith("__") and _os.path.exists(_os.path.join(_os.path.dirname(__file__), name + ".py")):
        value = importlib.import_module("." + name, __name__)     # find_circ2_amd.<submodule>
    else:
        raise AttributeError("module 'find_circ2_amd' has no attribute %r" % (name,))
    globals()[name] = value
    return value


__version__ = "0.1.0"

__all__ = ["Genome", "Options", "PairBatch", "ScanOutput", "Splice", "SynthConfig", "JunctionSpan", "reorder",
           "BreakpointEngine", "BreakpointError", "scan", "decode_splices", "first_tie_arrays", "gtag_str",
           "sq_table", "synthetic_n_intervals", "splices_or_raise", "CompactResults", "compact", "expand"]
