"""ctypes binding of libfc2.so (C ABI in include/fc2_bp.h).

The library is built in-tree (``find_circ2_amd/libfc2.so``) by
``__graft_entry__.build()`` / ``make -C find_circ2_amd/csrc``.  There is no
fallback: if the library is missing, importing a GPU entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

from ._lazy import LazyModule
from ._libpath import LIB_PATH, _HERE

np = LazyModule("numpy", globals(), "np")

FC2_OK = 0
CALLER_MAX_QUEUED = 64      # FC2_CALLER_MAX_QUEUED (include/fc2_caller.h): chunks fc2_caller_next keeps queued
FC2_E_PARAM = -1
FC2_E_HIP = -2
FC2_E_FORMAT = -3
FC2_E_RANGE = -4
FC2_E_IO = -5
FC2_E_KEY = -6
FC2_E_OS = -7

MAX_READ_LEN = 32767          # FC2_MAX_READ_LEN: longest read_part (x < 2^15 fits best_x, 2(l+1) ties fit n_ties)

PAIR_BACKSPLICE = 0x01
PAIR_PRIMARY_REV = 0x02
PAIR_READ_N = 0x04
PAIR_BYTEPATH = 0x08
PAIR_SKIP = 0x10
PAIR_WIN_N = 0x20
PAIR_READ_N1 = 0x40

RES_MINUS = 0x0001
RES_GTAG_SHIFT = 1
RES_GTAG_MASK = 0x1FFE
RES_ERR_KEY = 0x2000
RES_ERR_WIN = 0x4000
RES_DONE = 0x8000

_DTYPE_NAMES = ("PAIR_DTYPE", "RESULT_DTYPE", "ESCAPE_DTYPE", "LONG_PAIR_DTYPE", "LONG_RESULT_DTYPE")


def _dtypes():
    """The numpy record types of the C structs, made (and numpy imported) on first use."""
    PAIR_DTYPE = np.dtype([("a_pos", "<i4"), ("b_aend", "<i4"), ("chrom", "<u4"), ("read_len", "<u2"),
                           ("flags", "u1"), ("npos", "u1")])
    RESULT_DTYPE = np.dtype([("best_x", "<i2"), ("dist", "u1"), ("ov", "u1"), ("n_ties", "<u2"), ("info", "<u2")])
    assert PAIR_DTYPE.itemsize == 16 and RESULT_DTYPE.itemsize == 8
    ESCAPE_DTYPE = np.dtype([("index", "<u8"), ("result", RESULT_DTYPE)])     # fc2_result_escape
    # pairs with read parts over MAX_READ_LEN and their results (fc2_long_pair / fc2_long_result)
    LONG_PAIR_DTYPE = np.dtype([("read_off", "<u8"), ("read_len", "<u4"), ("chrom", "<u4"), ("a_pos", "<i4"),
                                ("b_aend", "<i4"), ("flags", "u1"), ("_pad", "u1", (7,))])
    LONG_RESULT_DTYPE = np.dtype([("best_x", "<i4"), ("n_ties", "<u4"), ("dist", "u1"), ("ov", "u1"), ("info", "<u2"),
                                  ("_pad", "<u4")])
    assert LONG_PAIR_DTYPE.itemsize == 32 and LONG_RESULT_DTYPE.itemsize == 16
    g = globals()
    for k in _DTYPE_NAMES:
        g[k] = locals()[k]


def __getattr__(name):
    if name in _DTYPE_NAMES:
        _dtypes()
        return globals()[name]
    raise AttributeError("module %r has no attribute %r" % (__name__, name))
R32_ESCAPE = 0x80000000
R16_ESCAPE = 0x007F


class Fc2Error(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("libfc2 error %d: %s" % (code, msg))
        self.code = code


class Params(ctypes.Structure):
    """``fc2_params``: the options find_breakpoints reads (find_circ.py:393-404)."""
    _fields_ = [("asize", ctypes.c_int32), ("margin", ctypes.c_int32), ("maxdist", ctypes.c_int32),
                ("noncanonical", ctypes.c_uint8), ("strandpref", ctypes.c_uint8),
                ("allhits", ctypes.c_uint8), ("_pad", ctypes.c_uint8)]


class GenomeView(ctypes.Structure):
    _fields_ = [("units", ctypes.c_void_p), ("nplane", ctypes.c_void_p), ("ncoarse", ctypes.c_void_p),
                ("chrom_start", ctypes.c_void_p), ("chrom_size", ctypes.c_void_p),
                ("n_units", ctypes.c_uint64), ("n_chrom", ctypes.c_uint32), ("dummy", ctypes.c_uint32),
                ("units_twin", ctypes.c_void_p), ("nsuper", ctypes.c_void_p), ("nsuper_shift", ctypes.c_uint32),
                ("nsuper_words", ctypes.c_uint32), ("wt", ctypes.c_void_p), ("wt_bytes", ctypes.c_uint64),
                ("wt_twin_off", ctypes.c_uint64)]


class BatchView(ctypes.Structure):
    _fields_ = [("pairs", ctypes.c_void_p), ("read_words", ctypes.c_void_p), ("read_nwords", ctypes.c_void_p),
                ("n", ctypes.c_uint64), ("stride", ctypes.c_uint64), ("rw", ctypes.c_uint32),
                ("nw", ctypes.c_uint32), ("max_l", ctypes.c_int32), ("layout", ctypes.c_uint32),
                ("win_words", ctypes.c_void_p), ("win_nwords", ctypes.c_void_p), ("ww", ctypes.c_uint32),
                ("wnw", ctypes.c_uint32)]


BATCH_LOCUS_ORDERED = 0x1
# per-call form hints (fc2_batch_view.layout, include/fc2_bp.h); results never depend on them
BATCH_FORM_STAGED = 0x02
BATCH_FORM_PLAIN = 0x04
BATCH_FORM_UNITS = 0x08
BATCH_FORM_TWOLANE = 0x10
BATCH_FORM_TRI = 0x20
BATCH_FORM_FIVE = 0x40
BATCH_FORM_WAVE = 0x80     # BASELINE north_star shape: one wavefront per pair (include/fc2_bp.h)


class CompactOut(ctypes.Structure):        # fc2_compact_out
    _fields_ = [("width", ctypes.c_int32), ("esc_cap", ctypes.c_uint32), ("words", ctypes.c_void_p),
                ("esc", ctypes.c_void_p), ("esc_count", ctypes.c_void_p), ("count_out", ctypes.c_void_p)]


class ReorderInfo(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("workspace_bytes", ctypes.c_uint64), ("shift", ctypes.c_uint32),
                ("n_buckets", ctypes.c_uint32), ("bucket_bits", ctypes.c_uint32), ("n_chunks", ctypes.c_uint32),
                ("n_groups", ctypes.c_uint32), ("chunk", ctypes.c_uint32)]


class BytesView(ctypes.Structure):
    _fields_ = [("index", ctypes.c_void_p), ("pairs", ctypes.c_void_p), ("arena", ctypes.c_void_p),
                ("off", ctypes.c_void_p), ("m", ctypes.c_uint64)]


class SynthCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("len_min", ctypes.c_int32), ("len_max", ctypes.c_int32),
                ("p_planted", ctypes.c_float), ("p_minus_site", ctypes.c_float),
                ("p_backsplice", ctypes.c_float), ("mut_rate", ctypes.c_float), ("n_rate", ctypes.c_float),
                ("p_clip", ctypes.c_float), ("span_min", ctypes.c_int32), ("span_max", ctypes.c_int32),
                ("locus_ordered", ctypes.c_int32), ("p_three_seg", ctypes.c_float), ("first", ctypes.c_uint64)]


# every symbol include/fc2_bp.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "fc2_abi_version", "fc2_last_error", "fc2_device_count", "fc2_host_register", "fc2_host_unregister", "fc2_set_tuning", "fc2_get_tuning", "fc2_max_fast_l",
    "fc2_batch_geometry",
    "fc2_bp_scan_launch", "fc2_bp_scan_bytes_launch", "fc2_probe_pattern_launch",
    "fc2_result_compact_launch", "fc2_result_expand", "fc2_bp_scan_compact_launch", "fc2_host_device_pointer",
    "fc2_fasta_open", "fc2_fasta_close", "fc2_fasta_n_chrom", "fc2_fasta_chrom", "fc2_fasta_find",
    "fc2_fasta_get_upper", "fc2_fasta_layout", "fc2_fasta_pack", "fc2_fasta_prepack",
    "fc2_pack_pairs", "fc2_bytepath_size", "fc2_bytepath_fill", "fc2_window_geometry", "fc2_pack_windows",
    "fc2_gather_windows_launch", "fc2_long_geometry", "fc2_long_fill", "fc2_bp_scan_long_launch",
    "fc2_synth_genome_launch", "fc2_coarse_launch", "fc2_twin_launch", "fc2_wtab_geometry", "fc2_wtab_launch",
    "fc2_nsuper_geometry", "fc2_nsuper_launch", "fc2_synth_pairs_launch",
    "fc2_reorder_plan", "fc2_reorder_launch",
    # include/fc2_ingest.h
    "fc2_ingest_open", "fc2_ingest_close", "fc2_ingest_n_refs", "fc2_ingest_ref_name", "fc2_ingest_header",
    "fc2_ingest_next", "fc2_ingest_counts_get", "fc2_ingest_set_bam_out", "fc2_ingest_close_bam_out",
    "fc2_ingest_format", "fc2_sam_to_bam", "fc2_bgzf_inflate_launch",
    "fc2_ingest_set_gpu_inflate", "fc2_ingest_set_gpu_inflate_from", "fc2_ingest_inflate_counts",
    # include/fc2_caller.h
    "fc2_caller_open", "fc2_caller_set_genome", "fc2_caller_inflate_counts", "fc2_caller_ingest", "fc2_caller_close", "fc2_caller_next",
    "fc2_caller_submit", "fc2_caller_submit_compact", "fc2_caller_submit_long", "fc2_caller_queued", "fc2_caller_take", "fc2_caller_rows", "fc2_caller_write_rows", "fc2_caller_counter", "fc2_caller_stats",
    "fc2_caller_set_reads_gz", "fc2_caller_close_reads",
    # include/fc2_ctx.h
    "fc2_ctx_create", "fc2_ctx_create_sibling", "fc2_ctx_destroy", "fc2_ctx_genome_load", "fc2_ctx_genome_view", "fc2_ctx_scan_async",
    "fc2_ctx_sync", "fc2_ctx_scan_long", "fc2_ctx_stream", "fc2_ctx_last_error",
]


class IngestParams(ctypes.Structure):
    _fields_ = [("asize", ctypes.c_int32), ("nolinear", ctypes.c_uint8), ("noop", ctypes.c_uint8),
                ("_pad", ctypes.c_uint8 * 2)]


class IngestCounts(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_uint64), ("total_mates", ctypes.c_uint64), ("unmapped_reads", ctypes.c_uint64),
                ("unspliced_mates", ctypes.c_uint64), ("seg_too_short_skip", ctypes.c_uint64),
                ("records", ctypes.c_uint64), ("handed_back", ctypes.c_uint64)]

class CallerOpts(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("known_circ", ctypes.c_char_p), ("known_lin", ctypes.c_char_p),
                ("min_uniq_qual", ctypes.c_int32), ("asize", ctypes.c_int32), ("margin", ctypes.c_int32),
                ("maxdist", ctypes.c_int32), ("short_threshold", ctypes.c_int32), ("huge_threshold", ctypes.c_int32),
                ("noncanonical", ctypes.c_uint8), ("allhits", ctypes.c_uint8), ("stranded", ctypes.c_uint8),
                ("strandpref", ctypes.c_uint8), ("halfunique", ctypes.c_uint8), ("report_nobridges", ctypes.c_uint8),
                ("test", ctypes.c_uint8), ("nolinear", ctypes.c_uint8), ("multi_events", ctypes.c_uint8),
                ("noop", ctypes.c_uint8), ("write_reads", ctypes.c_uint8), ("write_multi", ctypes.c_uint8),
                ("_pad", ctypes.c_uint32), ("chunksize", ctypes.c_uint64)]


class CallerBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("reads", ctypes.c_void_p), ("read_off", ctypes.c_void_p),
                ("pairs", ctypes.c_void_p), ("n_long", ctypes.c_uint64), ("long_pairs", ctypes.c_void_p)]


_lib = None


def build(force: bool = False) -> str:
    srcdir = os.path.join(_HERE, "csrc")
    srcs = [os.path.join(srcdir, f) for f in ("fc2_kernels.hip", "fc2_scan32.hip", "fc2_reorder.hip", "fc2_inflate.hip",
                                              "fc2_scan32.h",
                                              "fc2_host.cpp", "fc2_ingest.cpp", "fc2_ingest_impl.h", "fc2_caller.cpp",
                                              "fc2_bamout.cpp", "fc2_bamout.h", "fc2_ctx.cpp", "fc2_hostmem.h",
                                              "fc2_common.h", "Makefile")]
    srcs += [os.path.join(os.path.dirname(_HERE), "include", h)
             for h in ("fc2_bp.h", "fc2_ingest.h", "fc2_caller.h", "fc2_ctx.h")]
    newest = max(os.path.getmtime(s) for s in srcs)
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        subprocess.check_call(["make", "-s", "-C", srcdir])
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libfc2.so is not built (%s); run __graft_entry__.build() -- there is no CPU fallback"
                          % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, i32, i64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int64
    P = ctypes.POINTER
    sig = {
        "fc2_abi_version": (ctypes.c_int, []),
        "fc2_last_error": (ctypes.c_char_p, []),
        "fc2_device_count": (ctypes.c_int, [P(ctypes.c_int)]),
        "fc2_max_fast_l": (ctypes.c_int, []),
        "fc2_host_register": (ctypes.c_int, [vp, u64]),
        "fc2_host_unregister": (ctypes.c_int, [vp]),
        "fc2_set_tuning": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
        "fc2_get_tuning": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
        "fc2_batch_geometry": (ctypes.c_int, [P(Params), i32, P(u32), P(u32), P(u32)]),
        "fc2_bp_scan_launch": (ctypes.c_int, [P(Params), P(GenomeView), P(BatchView), vp, vp, u32, vp]),
        "fc2_bp_scan_bytes_launch": (ctypes.c_int, [P(Params), P(BytesView), vp, vp, u32, u64, vp]),
        "fc2_probe_pattern_launch": (ctypes.c_int, [P(Params), P(GenomeView), P(BatchView), vp, vp]),
        "fc2_result_compact_launch": (ctypes.c_int, [P(Params), vp, u64, ctypes.c_int, vp, vp, u32, vp, vp]),
        "fc2_result_expand": (ctypes.c_int, [P(Params), vp, ctypes.c_int, u64, vp, u64, vp, ctypes.c_int]),
        "fc2_bp_scan_compact_launch": (ctypes.c_int, [P(Params), P(GenomeView), P(BatchView), P(CompactOut), vp]),
        "fc2_host_device_pointer": (ctypes.c_int, [vp, P(vp)]),
        "fc2_fasta_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, P(vp)]),
        "fc2_fasta_close": (None, [vp]),
        "fc2_fasta_n_chrom": (ctypes.c_int, [vp]),
        "fc2_fasta_chrom": (ctypes.c_int, [vp, ctypes.c_int, P(ctypes.c_char_p), P(i64), P(i64), P(i64),
                                           P(i64), P(ctypes.c_int)]),
        "fc2_fasta_find": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "fc2_fasta_get_upper": (ctypes.c_int, [vp, ctypes.c_int, i64, i64, vp, i64, P(i64)]),
        "fc2_fasta_layout": (ctypes.c_int, [vp, P(u64), P(u64), vp]),
        "fc2_fasta_pack": (ctypes.c_int, [vp, vp, vp, vp, P(u64), ctypes.c_int]),
        "fc2_fasta_prepack": (ctypes.c_int, [vp, ctypes.c_int]),
        "fc2_pack_pairs": (ctypes.c_int, [P(Params), vp, u64, vp, vp, vp, vp, u32, vp, u32, u64, P(u64),
                                          ctypes.c_int]),
        "fc2_bytepath_size": (ctypes.c_int, [P(Params), u64, vp, P(u64), P(u64)]),
        "fc2_window_geometry": (ctypes.c_int, [P(Params), ctypes.c_int, P(u32), P(u32), P(u32)]),
        "fc2_pack_windows": (ctypes.c_int, [P(Params), vp, u64, vp, vp, vp, u32, u64, ctypes.c_int]),
        "fc2_gather_windows_launch": (ctypes.c_int, [P(Params), P(GenomeView), P(BatchView), vp, vp, vp, u32, vp]),
        "fc2_bytepath_fill": (ctypes.c_int, [P(Params), vp, u64, vp, vp, vp, vp, vp, vp, vp]),
        "fc2_long_geometry": (ctypes.c_int, [P(Params), u64, vp, P(ctypes.c_uint64), vp]),
        "fc2_long_fill": (ctypes.c_int, [P(Params), vp, u64, vp, vp, vp, vp]),
        "fc2_bp_scan_long_launch": (ctypes.c_int, [P(Params), u64, vp, vp, vp, vp, vp, vp, vp]),
        "fc2_synth_genome_launch": (ctypes.c_int, [u64, vp, vp, vp, u64, vp, vp, u32, vp]),
        "fc2_coarse_launch": (ctypes.c_int, [vp, vp, u64, vp]),
        "fc2_twin_launch": (ctypes.c_int, [vp, u64, vp, vp]),
        "fc2_wtab_geometry": (ctypes.c_int, [u64, P(u64), P(u64)]),
        "fc2_wtab_launch": (ctypes.c_int, [vp, u64, vp, vp]),
        "fc2_nsuper_geometry": (ctypes.c_int, [u64, P(u32), P(u32)]),
        "fc2_nsuper_launch": (ctypes.c_int, [vp, u64, vp, vp]),
        "fc2_synth_pairs_launch": (ctypes.c_int, [P(Params), P(SynthCfg), P(GenomeView), vp, u64, vp, vp, u32,
                                                  vp, u32, u64, vp, vp]),
        "fc2_reorder_plan": (ctypes.c_int, [P(GenomeView), u64, P(ReorderInfo)]),
        "fc2_reorder_launch": (ctypes.c_int, [P(ReorderInfo), P(GenomeView), P(BatchView), vp, vp, vp, vp, vp, vp]),
        "fc2_ingest_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, P(vp)]),
        "fc2_ingest_close": (None, [vp]),
        "fc2_ingest_n_refs": (ctypes.c_int, [vp]),
        "fc2_ingest_ref_name": (ctypes.c_char_p, [vp, ctypes.c_int]),
        "fc2_ingest_header": (ctypes.c_char_p, [vp]),
        "fc2_ingest_next": (ctypes.c_int, [vp, P(IngestParams), u64, P(IngestCounts), P(ctypes.c_void_p), P(u64),
                                           P(u64), P(ctypes.c_int)]),
        "fc2_ingest_counts_get": (ctypes.c_int, [vp, P(IngestCounts)]),
        "fc2_ingest_set_bam_out": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "fc2_ingest_close_bam_out": (ctypes.c_int, [vp]),
        "fc2_ingest_format": (ctypes.c_int, [vp, P(ctypes.c_int)]),
        "fc2_sam_to_bam": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p]),
        "fc2_caller_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, P(CallerOpts), P(vp)]),
        "fc2_caller_set_genome": (ctypes.c_int, [vp, vp, i32, vp, P(u64), P(u64)]),
        "fc2_caller_ingest": (vp, [vp]),
        "fc2_caller_close": (None, [vp]),
        "fc2_caller_next": (ctypes.c_int, [vp, P(CallerBatch), P(ctypes.c_int)]),
        "fc2_caller_submit": (ctypes.c_int, [vp, vp, vp, u32, u64]),
        "fc2_caller_submit_compact": (ctypes.c_int, [vp, vp, ctypes.c_int, u64, vp, u64, vp, u32, u64]),
        "fc2_caller_submit_long": (ctypes.c_int, [vp, vp, u64, vp, u64]),
        "fc2_caller_queued": (ctypes.c_int, [vp]),
        "fc2_caller_take": (ctypes.c_int, [vp, ctypes.c_int, P(ctypes.c_void_p), P(u64)]),
        "fc2_caller_set_reads_gz": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, u64]),
        "fc2_caller_close_reads": (ctypes.c_int, [vp]),
        "fc2_caller_rows": (ctypes.c_int, [vp, ctypes.c_int, P(ctypes.c_void_p), P(u64)]),
        "fc2_caller_write_rows": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, P(u64)]),
        "fc2_caller_counter": (ctypes.c_int, [vp, ctypes.c_int, P(ctypes.c_char_p), P(ctypes.c_double)]),
        "fc2_caller_stats": (ctypes.c_int, [vp, P(u64), P(u64)]),
        "fc2_bgzf_inflate_launch": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, u32, vp]),
        "fc2_ingest_set_gpu_inflate": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int]),
        "fc2_ingest_set_gpu_inflate_from": (ctypes.c_int, [vp, ctypes.c_int, u64]),
        "fc2_ingest_inflate_counts": (ctypes.c_int, [vp, P(u64), P(u64)]),
        "fc2_caller_inflate_counts": (ctypes.c_int, [vp, P(u64), P(u64)]),
        "fc2_ctx_create": (ctypes.c_int, [ctypes.c_int, P(vp)]),
        "fc2_ctx_create_sibling": (ctypes.c_int, [vp, P(vp)]),
        "fc2_ctx_destroy": (None, [vp]),
        "fc2_ctx_genome_load": (ctypes.c_int, [vp, vp, ctypes.c_int]),
        "fc2_ctx_genome_view": (ctypes.c_int, [vp, P(GenomeView)]),
        "fc2_ctx_scan_async": (ctypes.c_int, [vp, P(Params), u64, vp, vp, vp, vp, vp, u32, ctypes.c_int]),
        "fc2_ctx_sync": (ctypes.c_int, [vp]),
        "fc2_ctx_scan_long": (ctypes.c_int, [vp, P(Params), u64, vp, vp, vp, vp]),
        "fc2_ctx_stream": (vp, [vp]),
        "fc2_ctx_last_error": (ctypes.c_char_p, [vp]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("FC2_LIB_VARIANT") and not hasattr(L, name):
            continue              # an A/B build of an older revision may predate a symbol
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.fc2_abi_version() != 1:
        raise ImportError("libfc2.so ABI mismatch")
    _lib = L
    return L


def get_tuning(key: int) -> int:
    """Current value of an FC2_TUNE_* knob (fc2_get_tuning)."""
    v = ctypes.c_int(0)
    check(lib().fc2_get_tuning(key, ctypes.byref(v)))
    return v.value


def check(rc: int) -> None:
    if rc != FC2_OK:
        msg = lib().fc2_last_error()
        raise Fc2Error(rc, msg.decode("utf-8", "replace") if msg else "")


def ptr(a) -> int:
    """Address of a numpy array or torch tensor (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()
