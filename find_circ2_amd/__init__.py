"""find_circ2_amd -- MI355X-native breakpoint search for find_circ2.

One hot path of find_circ2 (find_circ.py 1.99), ``JunctionSpan.find_breakpoints``
plus its genome window fetch, as hand-written HIP kernels for gfx950 behind a
C ABI (include/fc2_bp.h, libfc2.so).  See DESIGN.md.
"""
from . import _native
from .genome import Genome, sq_table, synthetic_n_intervals
from .hotpath import (BreakpointEngine, BreakpointError, CompactResults, JunctionSpan, Options, PairBatch, ScanOutput,
                      Splice, SynthConfig, compact, decode_splices, expand, first_tie_arrays, gtag_str, reorder, scan,
                      splices_or_raise)

__version__ = "0.1.0"

__all__ = ["Genome", "Options", "PairBatch", "ScanOutput", "Splice", "SynthConfig", "JunctionSpan", "reorder",
           "BreakpointEngine", "BreakpointError", "scan", "decode_splices", "first_tie_arrays", "gtag_str",
           "sq_table", "synthetic_n_intervals", "splices_or_raise", "CompactResults", "compact", "expand"]
