"""The CLI's device genome, started before the package's imports (``python -m find_circ2_amd.cli``).

Interpreter start-up and ``import numpy`` take ~0.14 s of the CLI's process wall on the GPU box, and
making the genome resident ~0.2 s (HIP init, the 2-bit pack of the FASTA, the upload; DESIGN.md §5
"Start-up").  find_circ2_amd/__init__.py calls ``start`` first thing when the process runs the CLI
module: the command line is parsed with the CLI's own parser (cliopts) and, for the default native
loop, a thread opens the FASTA (.byo_index read or written, find_circ.py:110-115) and builds the same
contexts ``ctxpipe.CtxPipeline`` would -- a context per device with the resident genome, sibling
contexts sharing it -- through ctypes calls alone (they release the GIL), so the imports run meanwhile.
``cli.main`` adopts them (``take``): ``ctxpipe.FastaGenome.adopt`` and ``CtxPipeline(prestart=...)``,
which raise whatever opening the FASTA or building the contexts failed with, where the CLI raised it
before.  Nothing here runs for a library import, ``--help``, ``--version``, unparsable arguments, the
Python loops or a missing library: main then does all of it itself.
"""
import ctypes
import optparse
import os
import threading
import time

from ._libpath import LIB_PATH
from .cliopts import apply_threads, build_parser

FC2_OK = 0
FC2_E_IO = -5
PER_DEVICE = 2                      # contexts per device (CtxPipeline's default)

_started = None                     # this process's Prestart, until main takes it


class _Skip(Exception):
    pass


class _QuietParser(optparse.OptionParser):
    """The CLI's parser without output or exit: anything but a plain run is left to main()."""

    def exit(self, status=0, msg=None):
        raise _Skip()

    def error(self, msg):
        raise _Skip()

    def print_help(self, file=None):
        raise _Skip()

    def print_usage(self, file=None):
        raise _Skip()

    def print_version(self, file=None):
        raise _Skip()


def device_index(device) -> int:
    """'cuda:k' / 'hip:k' / k -> k (ctxpipe.device_index)."""
    s = str(device)
    return int(s.split(":", 1)[1]) if ":" in s else int(s)


class Prestart:
    """The FASTA handle and contexts built on a thread; ``key`` = the options they were built for."""

    def __init__(self, genome: str, device: str, gpus: int):
        self.key = (genome, device, gpus)
        self.fasta = None               # fc2_fasta* (int) or None (dummy mode / failed)
        self.dummy = False              # fc2_fasta_open raised the reference's IOError (FC2_E_IO)
        self.fasta_error = None         # (rc, message) of another fc2_fasta_open failure
        self.error = None               # (rc, message) of the device part (contexts already destroyed)
        self.ctxs = []                  # (fc2_ctx* int, device, primary) in CtxPipeline's order
        self.n_ctx = 0
        self.genome_index_s = self.hip_init_s = self.load_s = None
        self.genome_load_s = self.siblings_s = self.prepack_s = 0.0
        self.fasta_ready = threading.Event()
        self.taken = False
        self.thread = threading.Thread(target=self._run, name="fc2-genome-prestart", daemon=True)
        self.thread.start()

    def _run(self):
        try:
            self._build()
        except BaseException as ex:     # noqa: BLE001 -- kept for main
            if self.error is None and self.fasta_error is None:
                self.error = (-1, "genome prestart: %r" % (ex,))
        finally:
            self.fasta_ready.set()

    def _build(self):
        L = ctypes.CDLL(LIB_PATH)
        vp, P = ctypes.c_void_p, ctypes.POINTER
        for name, res, args in (("fc2_last_error", ctypes.c_char_p, []),
                                ("fc2_fasta_open", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, P(vp)]),
                                ("fc2_fasta_prepack", ctypes.c_int, [vp, ctypes.c_int]),
                                ("fc2_device_count", ctypes.c_int, [P(ctypes.c_int)]),
                                ("fc2_ctx_create", ctypes.c_int, [ctypes.c_int, P(vp)]),
                                ("fc2_ctx_create_sibling", ctypes.c_int, [vp, P(vp)]),
                                ("fc2_ctx_genome_load", ctypes.c_int, [vp, vp, ctypes.c_int]),
                                ("fc2_ctx_last_error", ctypes.c_char_p, [vp]),
                                ("fc2_ctx_destroy", None, [vp])):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args

        def last(msg):
            return msg.decode("utf-8", "replace") if msg else ""

        genome, device, gpus = self.key
        t = time.time()
        h = vp()
        rc = L.fc2_fasta_open(genome.encode(), 1, ctypes.byref(h))
        self.genome_index_s = time.time() - t
        if rc == FC2_E_IO:
            self.dummy = True
        elif rc != FC2_OK:
            self.fasta_error = (rc, last(L.fc2_last_error()))
            return
        else:
            self.fasta = h.value
        self.fasta_ready.set()
        t0 = time.time()
        made = []
        first_ctx = {}

        def first_context():
            """HIP initialisation (the device count for --gpus N, the first context) on a thread of its
            own while this one packs the FASTA's 2-bit planes (fc2_fasta_prepack)."""
            # cli._devices: --gpus N devices from --device on, wrapping round the devices present
            first = device_index(device)
            if gpus <= 1:
                devs = [first]
            else:
                n = ctypes.c_int(0)
                rc = L.fc2_device_count(ctypes.byref(n))
                if rc != FC2_OK:
                    first_ctx["error"] = (rc, last(L.fc2_last_error()))
                    return
                devs = [(first + k) % max(1, n.value) for k in range(gpus)]
            first_ctx["devs"] = devs
            c = vp()
            rc = L.fc2_ctx_create(devs[0], ctypes.byref(c))
            if rc != FC2_OK:
                first_ctx["error"] = (rc, last(L.fc2_last_error()))
                return
            first_ctx["ctx"] = c.value
            first_ctx["hip_init_s"] = time.time() - t0

        th = threading.Thread(target=first_context, name="fc2-hip-init", daemon=True)
        th.start()
        if self.fasta is not None:
            # two cores fewer than the pack would take (fc2_host.cpp n_workers): HIP's initialisation
            # and the interpreter's imports run meanwhile, and they are the longer path
            cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or os.cpu_count() or 1
            tp = time.time()
            L.fc2_fasta_prepack(self.fasta, max(1, min(cores, 64) - 2))   # (a failure shows again below)
            self.prepack_s = time.time() - tp
        th.join()
        try:
            if "error" in first_ctx:
                self.error = first_ctx["error"]
                return
            devs = first_ctx["devs"]
            self.hip_init_s = first_ctx["hip_init_s"]
            self.n_ctx = len(devs) * PER_DEVICE
            primary = {}
            for dev in devs:                       # CtxPipeline._build, call for call
                if dev not in primary:
                    c = vp()
                    if not made:
                        c.value = first_ctx["ctx"]
                    else:
                        rc = L.fc2_ctx_create(dev, ctypes.byref(c))
                        if rc != FC2_OK:
                            self.error = (rc, last(L.fc2_last_error()))
                            return
                    made.append((c.value, dev, True))
                    tg = time.time()
                    rc = L.fc2_ctx_genome_load(c, self.fasta, 0)
                    self.genome_load_s += time.time() - tg
                    if rc != FC2_OK:
                        self.error = (rc, last(L.fc2_ctx_last_error(c)))
                        return
                    primary[dev] = c.value
                    k0 = 1
                else:
                    k0 = 0
                for _ in range(k0, PER_DEVICE):
                    ts = time.time()
                    c = vp()
                    rc = L.fc2_ctx_create_sibling(primary[dev], ctypes.byref(c))
                    if rc != FC2_OK:
                        self.error = (rc, last(L.fc2_last_error()))
                        return
                    made.append((c.value, dev, False))
                    self.siblings_s += time.time() - ts
            self.ctxs = made
            self.load_s = time.time() - t0
        finally:
            if self.error is not None:             # siblings before the contexts whose genome they read
                for primary_pass in (False, True):
                    for h_, _, p in made:
                        if p == primary_pass:
                            L.fc2_ctx_destroy(h_)

    def discard(self):
        """Options differ from what was started (main builds its own): release everything."""
        self.thread.join()
        if os.path.exists(LIB_PATH):
            L = ctypes.CDLL(LIB_PATH)
            L.fc2_ctx_destroy.argtypes = [ctypes.c_void_p]
            L.fc2_fasta_close.argtypes = [ctypes.c_void_p]
            for primary_pass in (False, True):
                for h_, _, p in self.ctxs:
                    if p == primary_pass:
                        L.fc2_ctx_destroy(h_)
            if self.fasta is not None:
                L.fc2_fasta_close(self.fasta)
        self.ctxs, self.fasta = [], None


def start(argv) -> None:
    """From find_circ2_amd/__init__.py when the process runs ``python -m find_circ2_amd.cli``."""
    global _started
    if _started is not None or not os.path.exists(LIB_PATH):
        return
    try:
        options, _ = build_parser(_QuietParser).parse_args(list(argv))
    except _Skip:
        return
    if (options.version or options.system or not options.genome or options.python_ingest
            or options.python_caller):
        return
    apply_threads(options)
    try:
        device_index(options.device)
    except ValueError:
        return
    _started = Prestart(options.genome, options.device, options.gpus)


def take(options):
    """The prestart built for these options (once), else None; one built for others is discarded."""
    global _started
    p, _started = _started, None
    if p is None:
        return None
    if p.key != (options.genome, options.device, options.gpus):
        p.discard()
        return None
    p.taken = True
    return p
