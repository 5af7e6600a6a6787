#!/usr/bin/env python
"""Benchmark: anchor-pairs/s of the breakpoint search (find_circ.py:854-974) on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE
JSON line.  For N > 1 it runs under torch.distributed.run, one rank per GPU.

Workload (BASELINE.json configs[2] at N=1, configs[3] per GPU for N>1):
an hg19-shaped synthetic genome (the 93 @SQ contigs of test_data/test_norm.sam,
3.137 Gbp, ~7 % N runs) resident in HBM on every GPU, and per GPU a batch of
50M synthetic 100 bp backsplice anchor pairs (seeded).  A
"step" is one pass of the hot path over the GPU's batch: one find_breakpoints
evaluation per pair, genome window gather included.  Pairs are independent, so
ranks process their own shards with no collective on the data path (weak
scaling); the only collectives are the timing barrier and the max-over-ranks.

Also reported: ``roofline`` (the kernel's HBM fraction, its PMC traffic, and the ceiling of its
access pattern), ``cpu_baseline`` (the reference's path restated literally in Python, over a
process pool of the GPU's CPU share; 1-process and C legs in ``cpu_baseline_extra``),
``strong_scaling`` (configs[3]) and ``configs4_200M_150bp``; ``extra``: configs[1] (1M pairs on
CDR1as_locus.fa), the configs[4] per-GPU share, and the whole CLI in anchor pairs/s at 2M and 20M
reads (BAM on stdin).  ``--research`` adds the forms DESIGN.md §5 compares (pipelines, window-carrying,
wave-per-pair, reorder-then-scan, locus-ordered).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
STRONG_TAIL = 0          # configs[3]: default --strong-tail (shard.round_bounds)
CLI_RUNS = 3               # cli_end_to_end: BAM-on-stdin runs, the median reported
HEADLINE_RESULT_BYTES = 2  # the headline scan's result form: 2-byte compact words (fc2_bp_scan_compact_launch)
MERGE_ROUNDS = 5           # interleaved zero-copy / device-memory rounds behind merge_ms_per_step
METRIC = "anchor-pairs/sec (backsplice calls) at 100 bp reads, 1/2/4/8 MI355X"


def algo_bytes_per_pair(L: int, asize: int = 15, margin: int = 2, result_bytes: int = 8) -> int:
    """B(L) = ceil(l/4) + 2*ceil((l+2)/4) + 16 + R (2-bit read, two 2-bit windows,
    16 B record, R-byte result); 81 B at L = 100 with the 8-byte fc2_result, 75 B with the 2-byte
    compact word the headline scan writes (round 4)."""
    l = L - 2 * (asize - margin)
    return -(-l // 4) + 2 * (-(-(l + 2) // 4)) + 16 + result_bytes


def mean_algo_bytes(b, asize: int, margin: int) -> float:
    """B(L) of SURVEY.md 8(d) averaged over a batch's own read_part lengths (variable-length batches:
    configs[4]'s 120..150 bp reads and its shorter three-segment pairs)."""
    import torch
    L = b.pairs[:16 * b.n].view(b.n, 16)[:, 12:14].contiguous().view(torch.int16).to(torch.int64).flatten()
    l = L - 2 * (asize - margin)
    by = (l + 3) // 4 + 2 * ((l + 5) // 4) + 24
    return float(by.double().mean().item())


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["hg19", "cdr1as"], default="hg19")
    ap.add_argument("--pairs", type=int, default=0, help="pairs per GPU (default 50M hg19 / 1M cdr1as)")
    ap.add_argument("--read-len", type=int, default=100)
    ap.add_argument("--locus-ordered", dest="locus_ordered", action="store_true",
                    help="lay the batch out by A-window locus (PairBatch.pack(locus_order=True)); default read order")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the extras (configs[1], the configs[4] 150-bp share, the CLI end to end)")
    ap.add_argument("--research", action="store_true",
                    help="also run the research legs DESIGN.md §5 cites: device / host pipelines, window-carrying, "
                         "wave-per-pair and reorder-then-scan forms, the locus-ordered batch")
    ap.add_argument("--no-strong", action="store_true", help="skip the configs[3] strong-scaling / ordered-merge run")
    ap.add_argument("--no-config4", action="store_true", help="skip the configs[4] 200M x 120-150 bp run")
    ap.add_argument("--strong-batches", type=int, default=0,
                    help="configs[3]: batches per rank the stream is cut into (shard.round_robin_batch); 0: "
                         "max(2, 8 // ranks)")
    ap.add_argument("--strong-tail", type=int, default=-1,
                    help="configs[3]: cut each rank's last batch into t + 1 halving pieces (shard.round_bounds); "
                         "-1: the default, 0: equal batches")
    ap.add_argument("--config4-pairs", type=int, default=0, help="configs[4] stream length (default 200M; tests)")
    ap.add_argument("--no-cli", action="store_true", help="skip the end-to-end CLI extra (2M reads, BAM on stdin)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget per CPU baseline leg")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r06.json"))
    return ap.parse_args()


def setup_dist(args):
    """One process per GPU.  The hot path exchanges nothing between ranks, so the only
    collectives (timing barrier, max over ranks) run on a host gloo group by default;
    FC2_DIST_BACKEND=nccl selects RCCL instead.  With fewer GPUs than ranks (rehearsal
    on a 1-GPU box) ranks share devices round-robin."""
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    dev_index = local % ndev
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev_index)
        backend = os.environ.get("FC2_DIST_BACKEND", "gloo")
        # the process-group libraries log connection chatter on fd 1; keep stdout for the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
            else:
                dist.init_process_group("gloo")
            dist.barrier()
        finally:
            import ctypes
            ctypes.CDLL(None).fflush(None)   # C stdio buffers of the C++ libraries too
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return ws, rank, dev_index


def spawn_ranks(args) -> int:
    """``--gpus N`` without a launcher: start N rank processes of this script (one per GPU, the env
    torch.distributed.run would give them) BEFORE this process touches the GPU, forward rank 0's
    JSON line, and fail unless every rank finished and rank 0 reports n_gpus == N.  The parent
    never initialises HIP and never execs; it only waits on its children."""
    import socket
    import subprocess
    with socket.socket() as s:                  # a free rendezvous port on the loopback interface
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
    out0 = [b""]
    reader = threading.Thread(target=lambda: out0.__setitem__(0, procs[0].stdout.read()), daemon=True)
    reader.start()
    rcs = [None] * len(procs)
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            bad = [r for r, rc in enumerate(rcs) if rc not in (None, 0)]
            print("bench: rank(s) %s failed (exit %s); stopping the others" % (bad, [rcs[r] for r in bad]),
                  file=sys.stderr)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            return 1
        time.sleep(0.05)
    reader.join()
    lines = [l for l in out0[0].decode("utf-8", "replace").splitlines() if l.startswith("{")]
    if not lines:
        print("bench: rank 0 printed no JSON line", file=sys.stderr)
        return 1
    line = json.loads(lines[-1])
    if int(line.get("n_gpus", 0)) != args.gpus:
        print("bench: rank 0 reports n_gpus %s, asked for %d" % (line.get("n_gpus"), args.gpus), file=sys.stderr)
        return 1
    print(lines[-1], flush=True)
    return 0


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, ws: int, dev) -> float:
    from find_circ2_amd.shard import max_over_ranks as _mor   # gloo-tested helper (tests/test_shard_gloo.py)
    return x if ws == 1 else _mor(x, device=dev)


# 10 % three-segment reads (2 pairs each; their weight 0.5 is host-side only)
CONFIG5_THREE_SEG = 0.1


def workload_cfg(args, rank: int):
    """(pairs per GPU, SynthConfig keywords) of the workload: rank r's weak-scaling batch is the stream
    seeded 1337 + 7919 r; rank 0's stream is also configs[3]'s strong-scaling stream."""
    span = (150, 20000) if args.workload == "hg19" else (150, 2500)
    n = args.pairs or (50_000_000 if args.workload == "hg19" else 1_000_000)
    variable = bool(getattr(args, "read_len_min", None))      # configs[4]'s per-GPU share: config 5's reads
    kw = dict(seed=1337 + 7919 * rank, len_min=getattr(args, "read_len_min", None) or args.read_len,
              len_max=args.read_len, p_backsplice=1.0, p_planted=0.5, mut_rate=0.005, n_rate=0.0005,
              span_min=span[0], span_max=span[1], locus_ordered=bool(getattr(args, "locus_ordered", False)),
              p_three_seg=CONFIG5_THREE_SEG if variable else 0.0)
    return n, kw


def build_workload(args, rank, dev):
    from find_circ2_amd import Genome, Options, PairBatch, SynthConfig, sq_table
    opt = Options()
    if args.workload == "hg19":
        names, sizes = sq_table(os.path.join(GOLDEN, "test_norm.sam"))
        g = Genome.synthetic(names, sizes, seed=4711, device=dev)
    else:
        g = Genome.from_fasta(os.path.join(GOLDEN, "CDR1as_locus.fa"), device=dev)
    n, kw = workload_cfg(args, rank)
    b = PairBatch.synthetic(opt, g, n, SynthConfig(**kw))
    return opt, g, b


def device_pipeline(opt, g, b, reps: int, chunks: int = 8, width: int = 2):
    """BASELINE.md's 'device pipeline' number: pinned host SoA -> H2D -> scan -> D2H.

    The batch is split into `chunks` slices, each laid out contiguously in pinned
    host memory in the device SoA layout with its N rows in the sparse form PairBatch.pack
    uploads (hotpath.sparse_nrows; untimed setup), and streamed on two HIP
    streams so that one slice's copies overlap another's kernel (PCIe is full
    duplex).  The results come back in the 2-byte compact form (`width` 2: packed on the device by
    fc2_result_compact_launch, the slice's escape count and slots copied beside the words) or as
    the raw 8-byte words (`width` 8).  Returns pairs/s and ms per batch (median of `reps`); the
    check expands the compact words on the host (fc2_result_expand) and compares every result with
    the device-resident scan.
    """
    import torch
    from find_circ2_amd import CompactResults, PairBatch, compact, expand, scan
    from find_circ2_amd import _native as N
    from find_circ2_amd.hotpath import ScanOutput, scatter_nrows, widen_tail
    dev = b.device
    n = b.n
    step = (n + chunks - 1) // chunks
    words = b.read_words[:b.rw * b.stride].view(b.rw, b.stride)
    nwords = b.read_nwords[:b.nw * b.stride].view(b.nw, b.stride)
    flags = b.pairs[:16 * n].view(n, 16)[:, 14]
    narrow = b.rw > 1 and not bool((words[b.rw - 1] >> 32).any())
    host = []     # per slice: one pinned buffer [pairs | read rows but the last | last row (as uint32 when
                  # narrow) | N-row pair index | N rows of those pairs]
    for c in range(chunks):
        lo, hi = c * step, min(n, (c + 1) * step)
        if lo >= hi:
            break
        m = hi - lo
        # the N rows travel sparsely, as PairBatch.pack uploads them (hotpath.sparse_nrows)
        idx = torch.nonzero((flags[lo:hi] & N.PAIR_READ_N) != 0).flatten().to(torch.int64)
        # the last read row crosses as uint32 when it fits (hotpath.narrow_tail), as PairBatch.pack sends it
        tail = words[b.rw - 1, lo:hi].contiguous()
        if narrow:
            tail = tail.view(torch.int32)[0::2].contiguous()
            tail = torch.cat([tail, tail.new_zeros(m & 1)]).view(torch.int64)
        head = [b.pairs[16 * lo:16 * hi].view(torch.int64), words[:b.rw - 1, lo:hi].reshape(-1)]
        rest = [tail, idx, nwords[:, lo:hi][:, idx].reshape(-1)]
        hb = torch.cat([t.cpu() for t in head + rest]).pin_memory()
        host.append((lo, m, int(idx.numel()), (1 + b.rw) * m, hb))
    kmax = max(h[2] for h in host)
    if width not in (2, 8):
        raise ValueError("width is 2 or 8")
    cap = max(1024, step // 1024)
    host_out = torch.empty(n, dtype=torch.int64 if width == 8 else torch.int16).pin_memory()
    host_esc = torch.empty((chunks, 16 * (cap + 1)), dtype=torch.uint8).pin_memory()   # slots + count per slice
    dcomp = [CompactResults(step, dev, cap, width=2) for _ in range(2)] if width == 2 else None
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    tail_words = (step + 1) // 2 if narrow else step
    dbuf = [torch.empty((2 + b.rw) * step + tail_words + (1 + b.nw) * kmax, dtype=torch.int64, device=dev)
            for _ in range(2)]
    nbuf = [torch.zeros(b.nw * step, dtype=torch.int64, device=dev) for _ in range(2)]
    dres = [torch.empty(step, dtype=torch.int64, device=dev) for _ in range(2)]

    def slice_batch(buf, nb, m, k):
        sb = PairBatch()
        sb.options, sb.device = b.options, dev
        sb.rw, sb.nw, sb.tw, sb.max_l, sb.layout = b.rw, b.nw, b.tw, b.max_l, b.layout
        sb.n = sb.stride = m
        sb.pairs = buf[:2 * m].view(torch.uint8)
        sb.read_words = buf[2 * m:(2 + b.rw) * m]
        o = (2 + b.rw) * m                         # staging: last row | N-row index | N rows
        t2 = (m + 1) // 2 if narrow else m
        if narrow:
            widen_tail(sb.read_words[(b.rw - 1) * m:], buf[o:o + t2].view(torch.int32)[:m])
        else:
            sb.read_words[(b.rw - 1) * m:].copy_(buf[o:o + m])
        sb.read_nwords = nb[:b.nw * m]
        o += t2
        scatter_nrows(sb.read_nwords, buf[o:o + k], buf[o + k:o + k + b.nw * k].view(b.nw, k), b.nw, m)
        return sb

    def run_once():
        for c, (lo, m, k, nh, hbuf) in enumerate(host):
            st = streams[c & 1]
            with torch.cuda.stream(st):
                d = dbuf[c & 1]
                d[:nh].copy_(hbuf[:nh], non_blocking=True)                       # record + rows 0..rw-2
                d[nh + m:nh + m + hbuf.numel() - nh].copy_(hbuf[nh:], non_blocking=True)   # tail32 + N
                sb = slice_batch(d, nbuf[c & 1], m, k)
                scan(opt, g, sb, out=ScanOutput(dres[c & 1], None, sb.tw, m), stream=st.cuda_stream)
                if width == 8:
                    host_out[lo:lo + m].copy_(dres[c & 1][:m], non_blocking=True)
                else:
                    cr = compact(opt, dres[c & 1], m, into=dcomp[c & 1], stream=st.cuda_stream, width=2)
                    host_out[lo:lo + m].copy_(cr.words[:m], non_blocking=True)
                    host_esc[c].copy_(cr.esc_block.view(torch.uint8), non_blocking=True)
        torch.cuda.synchronize(dev)

    run_once()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run_once()
        ts.append(time.perf_counter() - t0)
    ms = float(np.median(ts)) * 1e3
    ok = None
    if hasattr(b, "_bench_ref_results"):
        if width == 8:
            ok = bool(torch.equal(host_out, b._bench_ref_results))
        else:
            words = host_out.numpy().view(np.uint16)
            esc = host_esc.numpy().view(N.ESCAPE_DTYPE)
            cnt = host_esc.numpy()[:, 16 * cap:16 * cap + 4].copy().view(np.int32)[:, 0]
            got = np.empty(n, np.int64)
            for c, (lo, m, _, _, _) in enumerate(host):
                k = int(cnt[c])
                if not 0 <= k <= cap:
                    raise RuntimeError("device pipeline slice %d: %d escapes, %d slots" % (c, k, cap))
                expand(opt, words[lo:lo + m], esc[c, :k], out=got[lo:lo + m])
            ok = bool(np.array_equal(got, b._bench_ref_results.numpy()))
    kn = sum(h[2] for h in host)
    h2d = sum(h[4].numel() * 8 for h in host)
    d2h = width * n + (0 if width == 8 else len(host) * 16 * (cap + 1))
    return {"value": round(n / (ms * 1e-3), 1), "unit": "anchor-pairs/s", "ms_per_batch": round(ms, 3),
            "pcie_GBs": round((h2d + d2h) / (ms * 1e-3) / 1e9, 1),
            "h2d_bytes_per_pair": round(h2d / n, 2), "d2h_bytes_per_pair": round(d2h / n, 2),
            "results_equal_device_resident_scan": ok,
            "note": "pinned host SoA (16 B record + %d B read rows%s; the N rows of the %.2f %% "
                    "of pairs flagged READ_N as index + %d B rows, scattered on the device) -> H2D -> bp_scan -> "
                    "D2H %s, %d slices on 2 HIP streams; %d pairs"
                    % (8 * b.rw - (4 if narrow else 0), ", the last one as uint32" if narrow else "",
                       100.0 * kn / max(n, 1), 8 * b.nw,
                       "8 B result" if width == 8 else "2 B compact result (+ escape slots, expanded on the host "
                       "for the check)", len(host), n)}


def host_read_arrays(opt, b, chunk: int = 4_000_000):
    """The batch as the read loop hands pairs out (fc2_caller_next): ASCII read_part bytes (anchors
    'A', the internal part decoded from the packed rows, 'N' from the N rows) at read_off[i] =
    i * max_len, and the 16-B records without the packer's flags.  Decoded on the device, untimed."""
    import torch
    from find_circ2_amd import _native as N
    dev = b.device
    n = b.n
    e = opt.eff_a
    hp = b.fetch_host_pairs().copy()
    has_n = torch.from_numpy((hp["flags"] & N.PAIR_READ_N) != 0).to(dev)
    hp["flags"] &= (N.PAIR_BACKSPLICE | N.PAIR_PRIMARY_REV | N.PAIR_SKIP)
    hp["npos"] = 0
    Lmax = int(hp["read_len"].max())
    reads = np.empty(n * Lmax + 16, np.uint8)
    code = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    W = b.read_words[:b.rw * b.stride].view(b.rw, b.stride)
    NW = b.read_nwords[:b.nw * b.stride].view(b.nw, b.stride)
    lens = torch.from_numpy(hp["read_len"].astype(np.int64)).to(dev)
    shifts = torch.arange(64, device=dev, dtype=torch.int64)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        m = hi - lo
        bits = ((W[:, lo:hi].t().unsqueeze(2) >> shifts) & 1).reshape(m, -1).to(torch.uint8)    # [m, rw*64]
        nbits = ((NW[:, lo:hi].t().unsqueeze(2) >> shifts) & 1).reshape(m, -1).to(torch.bool)
        l = (lens[lo:hi] - 2 * e).clamp(min=0)
        j = torch.arange(Lmax - 2 * e, device=dev).unsqueeze(0)
        jj = j.clamp(max=bits.shape[1] - 1).expand(m, -1)
        lob = torch.gather(bits, 1, jj)
        hib = torch.gather(bits, 1, (l.unsqueeze(1) + j).clamp(max=bits.shape[1] - 1))
        I = code[(lob | (hib << 1)).long()]
        I[torch.gather(nbits, 1, j.clamp(max=nbits.shape[1] - 1).expand(m, -1)) & has_n[lo:hi].unsqueeze(1)] = ord("N")
        out = torch.full((m, Lmax), ord("A"), dtype=torch.uint8, device=dev)
        out[:, e:Lmax - e] = I
        reads[lo * Lmax:hi * Lmax] = out.cpu().numpy().reshape(-1)
    reads[n * Lmax:] = 0
    off = np.arange(n, dtype=np.uint64) * np.uint64(Lmax)
    return reads, off, hp


def host_pipeline(opt, g, b, chunk: int = 4_000_000, reps: int = 3):
    """The product transfer path (find_circ2_amd.pipeline.ScanPipeline -- the Python loop's evaluator;
    the default CLI runs the same sequence inside libfc2.so, fc2_ctx_scan_async) from host pair arrays: per chunk the C++ packer writes records + read rows into
    page-locked staging, then async H2D, scan and D2H of the 8-B results on the scanner's side
    stream, two chunks in flight.  Timed from the host arrays to every raw result word in host
    memory in input order (what fc2_caller_submit consumes); must equal the device-resident scan."""
    from find_circ2_amd.pipeline import ScanPipeline
    reads, off, hp = host_read_arrays(opt, b)
    n = b.n
    pipe = ScanPipeline(g, opt)
    out = np.empty(n, np.int64)

    def run_once():
        pending = []
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            pending.append((lo, hi, pipe.submit(reads.ctypes.data, off[lo:hi], hp[lo:hi])))
            while len(pending) >= pipe.depth:
                a, z, t = pending.pop(0)
                out[a:z] = pipe.result(t, copy=False)[0]
        for a, z, t in pending:
            out[a:z] = pipe.result(t, copy=False)[0]

    run_once()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run_once()
        ts.append(time.perf_counter() - t0)
    s = float(np.median(ts))
    ok = bool(np.array_equal(out, b._bench_ref_results.numpy())) if hasattr(b, "_bench_ref_results") else None
    import os as _os
    return {"value": round(n / s, 1), "unit": "anchor-pairs/s", "ms_per_batch": round(s * 1e3, 1),
            "results_equal_device_resident_scan": ok, "chunk_pairs": chunk,
            "pack_threads": int(_os.environ.get("OMP_NUM_THREADS", "0") or 0) or "all cores (<= 64)",
            "note": "host pair arrays (read_part bytes + 16-B records, as fc2_caller_next hands them out) -> "
                    "C++ pack into pinned staging -> H2D -> scan -> D2H raw results, chunks of %d pairs, two per "
                    "side stream in flight (find_circ2_amd.pipeline; the CLI's fc2_ctx_scan_async does the same); median of %d passes "
                    "over %d pairs" % (chunk, reps, n)}


def stream_share(opt, g, cfg_kw, lo: int, hi: int):
    """Pairs [lo, hi) of a seeded synthetic stream, generated on this rank's device only (each pair
    depends on the seed and its stream index alone, fc2_synth_cfg.first): a rank holds its share of
    a stream, never the whole stream."""
    from find_circ2_amd import PairBatch, SynthConfig
    return PairBatch.synthetic(opt, g, hi - lo, SynthConfig(first=lo, **cfg_kw))


def results_checksum(res, first: int) -> int:
    """Order-sensitive checksum of result words res (device int64) at stream indices first..:
    sum over i of mix(word_i, index_i) mod 2^64, so shares of one stream add up to the whole."""
    import torch
    idx = torch.arange(first, first + res.numel(), device=res.device, dtype=torch.int64)
    h = res * -7046029254386353131 + idx * -4417276706812531889          # 0x9E37..., 0xC2B2... as int64
    h = h ^ ((h >> 29) & 0x7FFFFFFFF)
    return int(h.sum().item()) & 0xFFFFFFFFFFFFFFFF


def configs4(opt, g, ws, rank, dev, steps, warmup, total=200_000_000):
    """BASELINE configs[4]: ONE stream of `total` pairs of 120-150 bp reads (anchors of varying length,
    SURVEY.md 8(d) config 5, seed 4242), split into contiguous shares over the ranks -- total fixed
    (strong scaling); each rank generates and scans only its share on its resident hg19-shaped genome;
    value = total / max-over-ranks time.  At N = 1 one GPU holds and scans the whole stream (14 GB of
    SoA at 200M).  results_checksum: the stream's result words summed over the shares (order
    sensitive, shard-invariant): the same at every N."""
    import torch
    from find_circ2_amd.shard import gather_ints
    lo = total * rank // ws
    hi = total * (rank + 1) // ws
    n = hi - lo
    kw = dict(seed=4242, len_min=120, len_max=150, p_backsplice=1.0, p_planted=0.5, mut_rate=0.005, n_rate=0.0005,
              span_min=150, span_max=20000, p_three_seg=CONFIG5_THREE_SEG)
    b = stream_share(opt, g, kw, lo, hi)
    bmean = mean_algo_bytes(b, opt.asize, opt.margin)
    elapsed, kms, out = timed_scans(opt, g, b, steps, warmup, ws, dev)
    elapsed = max_over_ranks(elapsed, ws, dev)
    kms = max_over_ranks(kms, ws, dev)
    hits = int(((out.results[:n] & 0xFFFF) != 0xFFFF).sum())
    csum = sum(gather_ints(results_checksum(out.results[:n], lo))) & 0xFFFFFFFFFFFFFFFF
    del b, out
    torch.cuda.empty_cache()
    bpp = algo_bytes_per_pair(150, opt.asize, opt.margin)
    return {"value": round(total * steps / elapsed, 1), "unit": "anchor-pairs/s", "scaling": "strong",
            "ms_per_step": round(elapsed / steps * 1e3, 4), "kernel_ms_max_rank": round(kms, 4),
            "pairs_total": total, "pairs_per_rank": n, "ranks": ws, "rank0_pairs_with_hit": hits,
            "results_checksum": "%016x" % csum,
            "achieved_algo_GBs_per_rank_at_150bp": round(bpp * n / (kms * 1e-3) / 1e9, 1),
            "algo_bytes_per_pair_mean": round(bmean, 2),
            "achieved_algo_GBs_per_rank_at_mean": round(bmean * n / (kms * 1e-3) / 1e9, 1),
            "note": "configs[4]: one %d-pair stream (seed 4242), read lengths uniform in 120..150 bp, 10 %% of "
                    "pair slots the two anchor pairs of one three-segment read (SURVEY.md 8(d) config 5), cut into "
                    "contiguous shares over the ranks, each generated and scanned on its own rank's GPU; "
                    "hg19-shaped genome, read order; algorithmic bytes priced at 150 bp (%d B/pair) and at the "
                    "stream's mean read_part length" % (total, bpp)}


def reorder_then_scan(opt, g, b, steps, dev, bpp):
    """Locus order with its sort cost included: per step, the device locality reorder of the
    read-order batch (fc2_reorder_launch: a stable counting sort by genome bucket, find_circ2_amd.reorder)
    then the scan of the reordered copy; results mapped back to input order must equal the read-order scan."""
    import torch
    from find_circ2_amd import reorder, scan
    r = reorder(g, b)
    out = scan(opt, g, r)
    torch.cuda.synchronize(dev)
    slot = r.slot[:b.n].long()
    back = torch.empty_like(out.results[:b.n])
    back[slot] = out.results[:b.n]
    equal = bool(torch.equal(back.cpu(), b._bench_ref_results)) if hasattr(b, "_bench_ref_results") else None
    stream = torch.cuda.current_stream(dev)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e0, e1, e2 in ev:
        e0.record(stream)
        r = reorder(g, b, into=r)
        e1.record(stream)
        scan(opt, g, r, out=out, stream=stream.cuda_stream)
        e2.record(stream)
    torch.cuda.synchronize(dev)
    ro = float(np.mean([a.elapsed_time(m) for a, m, z in ev]))
    sc = float(np.mean([m.elapsed_time(z) for a, m, z in ev]))
    tot = ro + sc
    del r, out, back, slot
    torch.cuda.empty_cache()
    return {"value": round(b.n / (tot * 1e-3), 1), "unit": "anchor-pairs/s", "ms_per_step": round(tot, 4),
            "reorder_ms": round(ro, 4), "scan_ms": round(sc, 4),
            "frac_incl_sort": round(bpp * b.n / (tot * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_scan_only": round(bpp * b.n / (sc * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "results_equal_read_order_scan": equal,
            "note": "read-order batch reordered on the device by genome bucket, then scanned; both timed (HIP "
                    "events); the headline keeps the read-order scan because this sum is larger"}


def timed_scans(opt, g, b, steps, warmup, ws, dev, compact_width=0):
    """Warmup, then exactly `steps` scans bracketed by barrier + synchronize; per-launch HIP events.
    compact_width 2 / 4: the scans write their results in that compact form themselves
    (fc2_bp_scan_compact_launch into device memory, canonical mode), and after the timed region the
    words, expanded on the host, must equal the 8-byte scan's results word for word."""
    import torch
    from find_circ2_amd import CompactResults, scan
    from find_circ2_amd.hotpath import expand, scan_compact
    out = scan(opt, g, b)
    c = ctr = None
    if compact_width:
        c = CompactResults(b.n, dev, cap=max(1 << 16, b.n // 64), width=compact_width)
        ctr = torch.zeros(1, dtype=torch.int32, device=dev)

    def launch(stream=None):
        if c is None:
            scan(opt, g, b, out=out, stream=stream)
        else:
            scan_compact(opt, g, b, c.words.data_ptr(), c.width, c.esc.data_ptr(), c.cap, ctr.data_ptr(),
                         c.count.data_ptr(), stream=stream)
    for _ in range(max(0, warmup - 1)):
        launch()
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    barrier(ws)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(steps):
        ev[k][0].record(stream)
        launch(stream.cuda_stream)
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    barrier(ws)
    t1 = time.perf_counter()
    kms = [s.elapsed_time(e) for s, e in ev]
    if c is not None:                     # the compact words are the 8-byte results, exactly
        k = int(c.count.item())
        if k > c.cap:
            raise RuntimeError("compact headline: %d escapes, %d slots" % (k, c.cap))
        from find_circ2_amd import _native as N
        esc = c.esc.cpu().numpy().view(N.ESCAPE_DTYPE)[:k]
        words = c.words[:b.n].cpu().numpy()
        if not np.array_equal(expand(opt, words, esc), out.results[:b.n].cpu().numpy()):
            raise RuntimeError("compact headline: expanded words differ from the 8-byte scan")
    return t1 - t0, float(np.mean(kms)), out


def strong_scaling(opt, g, b0, ref64, ws, rank, dev, steps, warmup, n, cfg_kw, per_rank=4, streams=None, tail=0):
    """configs[3]: ONE pair stream (the `n` pairs rank 0 scans in the weak run, seed 1337) cut into
    contiguous batches dealt round-robin to the ranks (shard.my_batches).  Rank 0 scans views of its
    own weak batch; every other rank generates only its batches of the stream (stream_share).  Each
    batch's scan writes its results in the 2-byte transfer form (canonical mode) straight to the batch's
    input offset of ONE node-local page-locked host buffer (shard.SharedCompactResults) through the
    buffer's device address (fc2_bp_scan_compact_launch: the words cross PCIe as the scan's epilogue
    stores them), so rank 0 then holds every result in input order: the host-side ordered merge
    junction naming needs (find_circ.py:681-690, weights :544/:563/:579).  Timed: scans only; scans +
    that merge (with a barrier per step, so rank 0 could consume every step's merged results); and,
    for comparison, 8-byte scans whose results are packed to 2 or 4 bytes (fc2_result_compact_launch)
    or left at 8 bytes and copied D2H on a side stream.  Then checked passes: rank 0 poisons the buffer,
    every rank scans (and packs and copies), and the merged buffer expanded on the host
    (fc2_result_expand, what fc2_caller_submit_compact does
    per chunk) must equal rank 0's single-rank scan of the whole stream word for word (every form)."""
    import torch
    from find_circ2_amd import CompactResults, compact, scan
    from find_circ2_amd.hotpath import ScanOutput
    from find_circ2_amd.shard import (SharedCompactResults, SharedResults, broadcast_name, my_bounds, round_bounds,
                                      round_robin_batch)
    bsz = round_robin_batch(n, ws, per_rank=per_rank)
    bounds = round_bounds(n, ws, per_rank=per_rank, tail=tail)
    mine = my_bounds(bounds, rank, ws)
    cap = max(1024, bsz // 256)
    widths = (2, 4)
    if rank == 0:
        merged = {w: SharedCompactResults(n, bounds, cap, create=True, pin=True, width=w) for w in widths}
        raw = SharedResults(n, create=True, pin=True)
        names = [merged[w].name for w in widths] + [raw.name]
    names = broadcast_name(names if rank == 0 else None) if ws > 1 else names
    if rank != 0:
        merged = {w: SharedCompactResults(n, bounds, cap, name=names[k], pin=True, width=w)
                  for k, w in enumerate(widths)}
        raw = SharedResults(n, name=names[-1], pin=True)
    barrier(ws)                                  # every rank attached before rank 0 may unlink at the end
    subs = []
    for k, lo, hi in mine:
        s = b0.sub(lo, hi) if rank == 0 else stream_share(opt, g, cfg_kw, lo, hi)
        subs.append((k, lo, hi, s, torch.empty(hi - lo, dtype=torch.int64, device=dev),
                     {w: CompactResults(hi - lo, dev, cap, width=w) for w in widths}))
    # scans on one stream, the D2H of batch k on another, overlapping the scan of batch k+1
    stream, copier = streams if streams is not None else (torch.cuda.current_stream(dev), torch.cuda.Stream(dev))
    done = [torch.cuda.Event() for _ in subs]

    host = {"scan": 0.0, "copy": 0.0, "calls": 0}   # host seconds in the launch calls (FC2_BENCH_HOST_TIMING)
    clock = time.perf_counter if os.environ.get("FC2_BENCH_HOST_TIMING") else None

    # zero-copy form: the scan's epilogue writes each pair's 2-byte word straight into the shared
    # host buffer (fc2_bp_scan_compact_launch through the buffer's device address), escapes into the
    # batch's slots and the count into its slot: no 8-byte words, no pack launch, no copy
    from find_circ2_amd.hotpath import host_device_pointer, scan_compact
    zdev = host_device_pointer(merged[2].array.ctypes.data)
    zblk = 16 * (cap + 1)
    zctr = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in subs]

    def step(mode):                              # mode: None (scans only), 2, 4 (compact widths), 8 (raw), "z", "zd"
        if mode == "z":
            for j, (k, lo, hi, s, res, comp) in enumerate(subs):
                eb = zdev + merged[2]._w_bytes + k * zblk
                scan_compact(opt, g, s, zdev + 2 * lo, 2, eb, cap, zctr[j].data_ptr(), eb + 16 * cap,
                             stream=stream.cuda_stream)
            return
        if mode == "zd":                         # the same launches writing into device memory
            for j, (k, lo, hi, s, res, comp) in enumerate(subs):
                c = comp[2]
                scan_compact(opt, g, s, c.words.data_ptr(), 2, c.esc.data_ptr(), cap, zctr[j].data_ptr(),
                             c.count.data_ptr(), stream=stream.cuda_stream)
            return
        for j, (k, lo, hi, s, res, comp) in enumerate(subs):
            t0 = clock() if clock else 0.0
            scan(opt, g, s, out=ScanOutput(res, None, s.tw, s.stride), stream=stream.cuda_stream)
            if mode is None:
                continue
            if mode != 8:
                compact(opt, res, hi - lo, into=comp[mode], stream=stream.cuda_stream)
            done[j].record(stream)
            copier.wait_event(done[j])
            t1 = clock() if clock else 0.0
            with torch.cuda.stream(copier):
                if mode != 8:
                    m, c = merged[mode], comp[mode]
                    m.words_t[lo:hi].copy_(c.words[:hi - lo], non_blocking=True)
                    m.esc_t[k].copy_(c.esc_block.view(torch.uint8), non_blocking=True)   # slots + count
                else:
                    raw.tensor[lo:hi].copy_(res, non_blocking=True)
            if clock and mode == 2:
                t2 = clock()
                host["scan"] += t1 - t0
                host["copy"] += t2 - t1
                host["calls"] += 1
        if mode is not None:                     # the next step's scans overwrite res / comp
            stream.wait_stream(copier)

    def timed(mode) -> float:
        barrier(ws)
        t0 = time.perf_counter()
        for _ in range(steps):
            step(mode)
            if mode is not None:                 # rank 0 could consume this step's merged results
                torch.cuda.synchronize(dev)
                barrier(ws)
        torch.cuda.synchronize(dev)
        barrier(ws)
        return max_over_ranks(time.perf_counter() - t0, ws, dev)

    for mode in (2, 4, 8, "z", "zd"):
        for _ in range(max(1, warmup)):
            step(mode)
    torch.cuda.synchronize(dev)
    scan_s = timed(None)
    t = {mode: timed(mode) for mode in (2, 4, 8)}
    # the zero-copy merge against the same launches into device memory: interleaved rounds, paired
    # differences (a single pair of runs differs by +-0.03 ms per step from run-to-run noise alone)
    zz, zd = [], []
    for _ in range(MERGE_ROUNDS):
        zz.append(timed("z"))
        zd.append(timed("zd"))
    t["z"], t["zd"] = float(np.median(zz)), float(np.median(zd))
    merge_rounds = [round((a - b) / steps * 1e3, 4) for a, b in zip(zz, zd)]
    # checked passes, one per width (and the zero-copy form, which lands in the 2-byte buffer)
    equal, n_esc = {}, {}
    for w in widths + ("z",):
        m = merged[2 if w == "z" else w]
        if rank == 0:
            m.words[:] = 0x5A5A
            m.esc_count[:] = -1
        barrier(ws)
        step(w)
        torch.cuda.synchronize(dev)
        barrier(ws)
        if rank == 0:
            try:
                equal[w] = bool(np.array_equal(m.merged(opt), ref64))
                n_esc[w] = int(m.esc_count.sum())
            except Exception as ex:              # an overflowed escape area or a bad escape list
                equal[w], n_esc[w] = repr(ex), None
    out = None
    if rank == 0:
        def form(mode):
            return {"value": round(n * steps / t[mode], 1), "ms_per_step": round(t[mode] / steps * 1e3, 4),
                    "merge_ms_per_step": round((t[mode] - scan_s) / steps * 1e3, 4)}
        out = {
            "value": round(n * steps / t["z"], 1), "unit": "anchor-pairs/s", "scaling": "strong",
            "ms_per_step": round(t["z"] / steps * 1e3, 4),
            "scan_only": {"value": round(n * steps / scan_s, 1), "ms_per_step": round(scan_s / steps * 1e3, 4),
                          "note": "scans writing 8-byte results to HBM, no merge"},
            "scan_only_compact_device": {"value": round(n * steps / t["zd"], 1),
                                         "ms_per_step": round(t["zd"] / steps * 1e3, 4),
                                         "note": "the merge's own launches (fc2_bp_scan_compact_launch, 2-byte words, "
                                                 "escapes and count) writing into device memory, per-step barrier "
                                                 "as in the merge: the baseline of merge_ms_per_step"},
            "merge_ms_per_step": float(np.median(merge_rounds)),
            "merge_ms_per_step_rounds": merge_rounds,
            "merge_form": "zero_copy_2B: the scan's epilogue writes each pair's 2-byte word, the escapes and the "
                          "batch's escape count straight into the shared page-locked buffer through its device "
                          "address (fc2_bp_scan_compact_launch): no 8-byte results, pack launch or copy. "
                          "merge_ms_per_step = that run minus the same launches writing to device memory with the same "
                          "per-step barrier (scan_only_compact_device): the cost of the host destination alone; the "
                          "median of the paired differences of %d interleaved rounds (merge_ms_per_step_rounds)"
                          % MERGE_ROUNDS,
            "merge_bytes_per_pair": 2, "escapes": n_esc["z"],
            "merge_2B_copied": dict(form(2), escapes=n_esc[2], merged_equals_single_rank=equal[2],
                                    note="8-byte scan, pack launch, D2H copy on a side stream"),
            "merge_4B_words": dict(form(4), escapes=n_esc[4], merged_equals_single_rank=equal[4]),
            "merge_8B_words": form(8),
            "pairs_total": n, "batch_pairs": bsz, "n_batches": len(bounds), "ranks": ws, "tail_pieces": tail,
            "smallest_batch_pairs": min(hi - lo for lo, hi in bounds),
            "merged_equals_single_rank": equal["z"],
            **({"host_ms_per_batch_2B": {"scan_and_pack_launch": round(host["scan"] / max(1, host["calls"]) * 1e3, 4),
                                         "copy_calls": round(host["copy"] / max(1, host["calls"]) * 1e3, 4)}}
               if clock else {}),
            "note": "one %d-pair stream in %d contiguous batches of up to %d pairs dealt round-robin to %d rank(s) "
                    "(with tail_pieces = t, each rank's last batch cut into t + 1 halving pieces), each rank "
                    "holding only its batches; each batch's scan writes its results as 2-byte words (canonical "
                    "mode, escapes for the rest) straight into ONE node-local page-locked shared-memory buffer at "
                    "their input offsets (host-side ordered merge, no collective on the data path); value = stream "
                    "pairs / (scans + merge + per-step barrier), max over ranks; merge_2B_copied / merge_4B_words / "
                    "merge_8B_words = 8-byte scans whose results are packed (2 or 4 B) or not and copied D2H"
                    % (n, len(bounds), bsz, ws)}
    barrier(ws)
    for m in merged.values():
        m.close()
    raw.close()
    return out


# ---------------------------------------------------------------------------
# CPU baseline (oracle = test infrastructure, used ONLY as the reported baseline)
# ---------------------------------------------------------------------------
def _decode_sample(opt, g, b, idx):
    """Bytes of sampled pairs (internal read part padded with dummy anchors, both windows)."""
    import torch
    from find_circ2_amd import _native as N
    hp = b.fetch_host_pairs()[idx]
    e = opt.eff_a
    m = len(idx)
    W = b.read_words.view(b.rw, b.stride)[:, torch.as_tensor(idx, device=b.device)].cpu().numpy()
    bits = np.unpackbits(np.ascontiguousarray(W.T).view(np.uint8).reshape(m, -1), axis=1, bitorder="little")
    NWm = b.read_nwords.view(b.nw, b.stride)[:, torch.as_tensor(idx, device=b.device)].cpu().numpy()
    nbits = np.unpackbits(np.ascontiguousarray(NWm.T).view(np.uint8).reshape(m, -1), axis=1, bitorder="little")
    code = np.frombuffer(b"ACGTN", np.uint8)
    ls = hp["read_len"].astype(np.int64) - 2 * e
    lmax = int(ls.max())
    j = np.arange(lmax)[None, :]
    lo = np.take_along_axis(bits, np.minimum(j, bits.shape[1] - 1).repeat(m, 0), 1)
    hi = np.take_along_axis(bits, np.minimum(ls[:, None] + j, bits.shape[1] - 1), 1)
    I = code[(lo | (hi << 1)).astype(np.int64)]
    nmask = nbits[:, :lmax].astype(bool) & ((hp["flags"] & N.PAIR_READ_N) != 0)[:, None]
    I[nmask] = ord("N")
    U = g.units.cpu().numpy().view(np.uint64)
    NP = g.nplane.cpu().numpy().view(np.uint64)

    def windows(starts, lens):
        pos = starts[:, None] + np.arange(lens)[None, :]
        c = hp["chrom"].astype(np.int64)
        cs = g.chrom_start[c].astype(np.int64)[:, None]
        sz = g.sizes[c][:, None]
        inside = (pos >= 0) & (pos < sz)
        gp = np.where(inside, pos + cs, 0).astype(np.uint64)
        u = (gp >> np.uint64(6)).astype(np.int64)
        bb = gp & np.uint64(63)
        lo_ = (U[2 * u] >> bb) & np.uint64(1)
        hi_ = (U[2 * u + 1] >> bb) & np.uint64(1)
        nn = ((NP[u] >> bb) & np.uint64(1)).astype(bool) | ~inside
        w = code[(lo_ | (hi_ << np.uint64(1))).astype(np.int64)]
        w[nn] = ord("N")
        return w

    Lw = lmax + 2
    A = windows(hp["a_pos"].astype(np.int64) + e, Lw)
    B = windows(hp["b_aend"].astype(np.int64) - e - (ls + 2), Lw)
    reads, parts, woff = [], [], np.zeros(m, np.int64)
    pos = 0
    for k in range(m):
        lk = int(ls[k])
        reads.append(b"A" * e + I[k, :lk].tobytes() + b"A" * e)
        woff[k] = pos
        parts.append(A[k, :lk + 2].tobytes() + B[k, :lk + 2].tobytes())
        pos += 2 * (lk + 2)
    wins = np.frombuffer(b"".join(parts) + b"\0", np.uint8)
    return hp, reads, wins, woff, ls


def subset_fasta(g, d: str, k: int = 3):
    """The k largest chromosomes of the device genome written as a FASTA with 50-nt lines (as UCSC
    hg19) plus its .byo_index (fc2_fasta_open, the reference's store_index format,
    find_circ.py:157-179): the file the reference's Track/GenomeAccessor would mmap.  Decoded from
    the device planes in 16M-base pieces.  Returns (path, chromosome indices)."""
    import ctypes
    import torch
    from find_circ2_amd import _native as N
    order = [int(i) for i in np.argsort(-np.asarray(g.sizes, np.int64), kind="stable")[:k]]
    path = os.path.join(d, "subset.fa")
    code = torch.tensor(list(b"ACGTN"), dtype=torch.uint8, device=g.device)
    width = 50
    with open(path, "wb") as f:
        for c in order:
            f.write(b">" + g.names[c].encode() + b"\n")
            cs, size = int(g.chrom_start[c]), int(g.sizes[c])
            step = (1 << 24) // width * width
            for lo in range(0, size, step):
                hi = min(size, lo + step)
                pos = torch.arange(cs + lo, cs + hi, device=g.device, dtype=torch.int64)
                u, bit = pos >> 6, pos & 63
                lo_b = (g.units[2 * u] >> bit) & 1
                hi_b = (g.units[2 * u + 1] >> bit) & 1
                nn = (g.nplane[u] >> bit) & 1
                s = code[torch.where(nn == 1, 4, lo_b | (hi_b << 1))].cpu().numpy()
                full = len(s) // width
                f.write(np.concatenate([s[:full * width].reshape(full, width),
                                        np.full((full, 1), 10, np.uint8)], axis=1).tobytes())
                if len(s) % width:
                    f.write(s[full * width:].tobytes() + b"\n")
    h = ctypes.c_void_p()
    N.check(N.lib().fc2_fasta_open(path.encode(), 1, ctypes.byref(h)))     # writes subset.fa.byo_index
    N.lib().fc2_fasta_close(h)
    return path, order


def cpu_baselines(opt, g, b, budget_s):
    """The reported CPU baselines (never the target): (1) the reference's own per-pair path restated
    literally in Python -- find_breakpoints' O(l^2) string + numpy idiom (find_circ.py:854-974) with
    BOTH windows fetched per pair through Track.get -> GenomeAccessor.get_data -> indexed_fasta.get_data
    + .upper() (:900-902, :274-312, :362-368, :189-215) from an mmap'd FASTA of the bench genome (its
    three largest chromosomes, written from the device planes, with the .byo_index the reference
    loads), one core, on a sample of this batch's pairs on those chromosomes -- and its first ties
    checked against the GPU's results; (2) the C literal O(l^2) restatement, one core; (3) the C O(l)
    restatement on the box's CPU share, both on pre-decoded windows."""
    import shutil
    import tempfile
    import torch
    import oracle
    from oracle.bp_oracle import (Options as ROpt, RefGenomeTrack, RefIndexedFasta, Span,
                                  find_breakpoints as py_find)

    rng = np.random.default_rng(99)
    d = tempfile.mkdtemp(prefix="fc2_cpu_base_", dir="/tmp")
    try:
        t_fa = time.perf_counter()
        fa, subset = subset_fasta(g, d)
        fa_s = time.perf_counter() - t_fa
        chrom_col = b.pairs[:16 * b.n].view(torch.int32).view(b.n, 4)[:, 2]
        on_subset = torch.isin(chrom_col, torch.tensor(subset, dtype=torch.int32, device=b.device))
        cand = torch.nonzero(on_subset).flatten().cpu().numpy()
        n_sample = min(len(cand), 200_000)
        idx = np.sort(rng.choice(cand, n_sample, replace=False))
        hp, reads, wins, woff, ls = _decode_sample(opt, g, b, idx)
        bs = (hp["flags"] & 1) != 0
        rev = (hp["flags"] & 2) != 0
        skip = (hp["flags"] & 0x10) != 0
        gpu = b._bench_ref_results.numpy()[idx].view(np.uint64) if hasattr(b, "_bench_ref_results") else None

        # (1) the reference's path, literally: per pair two windows through the Track chain of an mmap'd
        # FASTA, then the per-x string concat + numpy compare
        track = RefGenomeTrack(RefIndexedFasta(fa, use_existing_index=True, use_mmap=True))
        ro = ROpt()
        done = agree = errors = 0
        t0 = time.perf_counter()
        for k in range(len(reads)):
            if skip[k]:
                continue
            # is_backsplice = B.pos - A.aend < 0 (find_circ.py:842): encode the flag through these two
            a_aend, b_pos = (1, 0) if bs[k] else (0, 1)
            sp = Span(g.names[int(hp["chrom"][k])], int(hp["a_pos"][k]), a_aend, b_pos, int(hp["b_aend"][k]),
                      reads[k], bool(rev[k]))
            try:
                ties = py_find(sp, track, ro)
                x = ties[0].x if ties else -1
                if gpu is not None:
                    gx = int(gpu[k] & np.uint64(0xFFFF))
                    gx = gx - 65536 if gx >= 32768 else gx
                    gt = int((gpu[k] >> np.uint64(32)) & np.uint64(0xFFFF))
                    agree += int(gx == x and gt == (ties[0].n_hits if ties else 0))
            except Exception:
                errors += 1
                agree += int(gpu is not None and int(gpu[k] >> np.uint64(48)) & 0x6000 != 0)
            done += 1
            if time.perf_counter() - t0 > budget_s:
                break
        py_rate = done / (time.perf_counter() - t0)
        # (1b) the same literal path on the host's cores: one spawned process per core of the GPU's CPU
        # share (each loads the FASTA through its own mmap + .byo_index, as separate reference processes
        # would), disjoint slices of the sample, every first tie checked against the GPU
        share = cpu_share()
        items = [k for k in range(len(reads)) if not skip[k]]
        spans = [(g.names[int(hp["chrom"][k])], int(hp["a_pos"][k]), *((1, 0) if bs[k] else (0, 1)),
                  int(hp["b_aend"][k]), reads[k], bool(rev[k])) for k in items]
        pool_res = None
        try:
            import multiprocessing as mp
            from oracle.bp_oracle import literal_rate
            P = share
            sl = [spans[len(spans) * i // P:len(spans) * (i + 1) // P] for i in range(P)]
            t_pool = time.perf_counter()
            with mp.get_context("spawn").Pool(P) as pool:
                outs = pool.starmap(literal_rate, [(fa, x, budget_s, True) for x in sl])
            wall_pool = time.perf_counter() - t_pool
            n_done = sum(o[0] for o in outs)
            pool_agree = pool_raised = 0
            for i, (nd, _, ties) in enumerate(outs):
                base = len(spans) * i // P
                for j, t in enumerate(ties):
                    k = items[base + j]
                    gw = int(gpu[k]) if gpu is not None else 0
                    if t is None:
                        pool_raised += 1
                        pool_agree += int((gw >> 48) & 0x6000 != 0)
                    else:
                        gx = gw & 0xFFFF
                        gx = gx - 65536 if gx >= 32768 else gx
                        pool_agree += int(gx == t[0] and ((gw >> 32) & 0xFFFF) == t[1])
            n_checked = sum(len(o[2]) for o in outs)
            pool_res = {"value": round(n_done / max(o[1] for o in outs), 1), "unit": "anchor-pairs/s",
                        "cores": P, "kind": "port", "pairs": n_done, "pairs_checked": n_checked,
                        "first_ties_agree_with_gpu": pool_agree,
                        "raised": pool_raised, "wall_s_incl_spawn": round(wall_pool, 1),
                        "per_process_pairs_per_s": round(n_done / P / max(o[1] for o in outs), 1)}
        except Exception as ex:         # an extra must not cost the bench line
            pool_res = {"error": repr(ex)}
    finally:
        shutil.rmtree(d, ignore_errors=True)

    # (2) C, literal O(l^2), one core;  (3) C, O(l), the box's CPU share (ctypes releases the GIL)
    p = oracle.params()

    def run_c(use_fast, lo, hi):
        return oracle.scan_windows(p, reads[lo:hi], wins, woff[lo:hi], hp["a_pos"][lo:hi], hp["b_aend"][lo:hi],
                                   bs[lo:hi], rev[lo:hi], use_fast=use_fast)

    t0 = time.perf_counter()
    k = 0
    chunk = 2000
    while k < len(reads) and time.perf_counter() - t0 < budget_s:
        run_c(False, k, min(len(reads), k + chunk))
        k += chunk
    naive_rate = min(k, len(reads)) / (time.perf_counter() - t0)
    visible = len(os.sched_getaffinity(0))
    cores = share
    t0 = time.perf_counter()
    done_fast = 0
    rounds = 0
    while time.perf_counter() - t0 < budget_s / 2 or rounds == 0:
        ths = []
        per = (len(reads) + cores - 1) // cores
        for c in range(cores):
            th = threading.Thread(target=run_c, args=(True, c * per, min(len(reads), (c + 1) * per)))
            th.start()
            ths.append(th)
        for th in ths:
            th.join()
        done_fast += len(reads)
        rounds += 1
    fast_rate = done_fast / (time.perf_counter() - t0)
    try:
        model = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":", 1)[1].strip()
    except Exception:
        model = "unknown"
    one_core = {"value": round(py_rate, 1), "unit": "anchor-pairs/s", "cores": 1, "kind": "port",
                "sample": "%d pairs, one process; first ties agree with the GPU on %d of %d (%d raised, as the "
                          "GPU flagged)" % (done, agree, done, errors)}
    sample = ("literal Python restatement of find_circ.py:854-974 (per-x string concat + numpy byte compare, "
              "oracle/bp_oracle.py) with both windows per pair fetched through Track.get -> "
              "GenomeAccessor.get_data -> indexed_fasta.get_data + .upper() (find_circ.py:900-902) from an "
              "mmap'd FASTA of the bench genome (%s, its 3 largest chromosomes; written with its .byo_index in "
              "%.1f s, untimed), on a sample of this batch's pairs there" % (",".join(g.names[c] for c in subset), fa_s))
    if pool_res and "value" in pool_res:
        main = dict(pool_res, sample="%d processes (one per core of the GPU's CPU share; %s) x %.0f s, each "
                                     "cycling over its slice: %s; first ties agree with the GPU on %d of %d distinct "
                                     "pairs (%d raised, as the GPU flagged); the 1-process rate: "
                                     "cpu_baseline_extra.python_1core"
                                     % (pool_res["cores"], cpu_model_note(visible), budget_s, sample,
                                        pool_res["first_ties_agree_with_gpu"], pool_res["pairs_checked"],
                                        pool_res["raised"]))
    else:
        main = dict(one_core, sample=one_core["sample"] + "; " + sample)
    return dict(
        main=main, python_1core=one_core, python_pool=pool_res,
        c_naive={"value": round(naive_rate, 1), "unit": "anchor-pairs/s", "cores": 1, "kind": "port",
                 "sample": "C literal O(l^2) restatement (oracle/bp_oracle.c) on the same sample, windows "
                           "pre-decoded"},
        c_fast={"value": round(fast_rate, 1), "unit": "anchor-pairs/s", "cores": cores, "kind": "port",
                "sample": "C O(l) prefix-sum restatement, %d threads (the GPU box's CPU share per GPU; "
                          "sched_getaffinity lists %d), %d pairs x %d rounds, windows pre-decoded" % (
                              cores, visible, len(reads), rounds)},
        cpu_model=model)


def cpu_share() -> int:
    """CPUs this process may use: the cgroup quota (cpu.max) when one is set, else the affinity set, at
    most 16 -- the GPU box grants 16 CPUs per GPU while sched_getaffinity lists the whole machine's."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 16))


def cpu_model_note(visible: int) -> str:
    try:
        model = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":", 1)[1].strip()
    except Exception:
        model = "unknown"
    return "%s, sched_getaffinity lists %d" % (model, visible)


def kernel_label(g, ordered: bool) -> str:
    """The bp_scan32 form fc2_bp_scan_launch picks for this batch (FC2_TUNE_STAGE auto rule)."""
    staged = (not ordered) and (not g.dummy) and g.n_units * 16 >= (64 << 20)
    words = g.wt is not None
    if staged:
        if words:
            return ("bp_scan32_stage_bt_kernel<512,NT> (one anchor pair per lane, 512-pair blocks; chromosome table "
                    "+ super-coarse N map in LDS; each window's 32 B of word pairs loaded by a lane pair in one "
                    "request, from whichever genome copy holds it inside one 128-B line)")
        return ("bp_scan32_kernel<4,NT,STAGE> (one anchor pair per lane; chromosome table + super-coarse N map in "
                "LDS; lane pairs load each window line with one L2 request)")
    return "bp_scan32_kernel<4,NT> (one anchor pair per lane%s)" % ("; word-pair windows" if words else "")


def pattern_ceiling(opt, g, b, dev, rounds: int = 5, reps: int = 4):
    """Speed of light of the read-order access pattern, live on this GPU: fc2_probe_pattern_launch
    replays the scan's memory traffic for this batch (same records, rows, window offsets and result
    stores) with none of its arithmetic.  Probe and scan launches are interleaved on one stream."""
    import ctypes
    import torch
    from find_circ2_amd import scan, _native as N
    if g.wt is None:
        return None
    stream = torch.cuda.current_stream(dev)
    junk = torch.empty(b.n, dtype=torch.int64, device=dev)
    gv, bv, pv = g.view(), b.view(), opt.params()
    out = scan(opt, g, b)
    probe, kern = [], []
    for _ in range(rounds):
        for which, acc in (("probe", probe), ("scan", kern)):
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record(stream)
            for _ in range(reps):
                if which == "probe":
                    N.check(N.lib().fc2_probe_pattern_launch(ctypes.byref(pv), ctypes.byref(gv), ctypes.byref(bv),
                                                             junk.data_ptr(), stream.cuda_stream))
                else:
                    scan(opt, g, b, out=out, stream=stream.cuda_stream)
            s1.record(stream)
            torch.cuda.synchronize(dev)
            acc.append(s0.elapsed_time(s1) / reps)
    pm, km = float(np.median(probe)), float(np.median(kern))
    return {"probe_ms": round(pm, 4), "scan_ms_same_run": round(km, 4), "scan_frac_of_ceiling": round(pm / km, 4),
            "source": "live: fc2_probe_pattern_launch replays this batch's memory pattern (NT-streamed records and "
                      "read rows, both windows' word pairs at the scan's offsets, 8-B result) without the search "
                      "arithmetic; %d interleaved rounds x %d launches, medians" % (rounds, reps)}


def window_carrying(opt, g, b, steps, dev, bpp):
    """North_star's form of the same workload: each pair's two windows travel with the batch
    (fc2_batch_view.win_words; on the host fc2_pack_windows reads them from the mmap'd FASTA, here
    fc2_gather_windows_launch builds the identical rows from the synthetic device genome, untimed)
    and the scan reads no genome -- it gets a view holding only the chromosome sizes.  Results must
    equal the gathering scan's."""
    import ctypes
    import torch
    from find_circ2_amd import scan, _native as N
    ref = scan(opt, g, b).results[:b.n].clone()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    b.carry_windows_from_device(g)
    t1.record()
    torch.cuda.synchronize(dev)
    gather_ms = t0.elapsed_time(t1)
    p = opt.params()
    gv = N.GenomeView(None, None, None, None, g.d_chrom_size.data_ptr(), 0, len(g.names), 0, None, None, 0, 0,
                      None, 0, 0)
    bv = b.view()
    res = torch.empty(b.stride, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch():
        N.check(N.lib().fc2_bp_scan_launch(ctypes.byref(p), ctypes.byref(gv), ctypes.byref(bv), res.data_ptr(),
                                           None, b.tw, stream.cuda_stream))
    launch()
    torch.cuda.synchronize(dev)
    equal = bool(torch.equal(res[:b.n], ref))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, z in ev:
        a.record(stream)
        launch()
        z.record(stream)
    torch.cuda.synchronize(dev)
    km = float(np.mean([a.elapsed_time(z) for a, z in ev]))
    moved = 16 + 8 * b.rw + 16 * b.pw + 8                 # record + read row + window rows + result
    ach = bpp * b.n / (km * 1e-3) / 1e9
    out = {"value": round(b.n / (km * 1e-3), 1), "unit": "anchor-pairs/s", "kernel_ms": round(km, 4),
           "achieved_algo_GBs": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
           "streamed_bytes_per_pair": moved,
           "streamed_GBs": round(moved * b.n / (km * 1e-3) / 1e9, 1),
           "results_equal_gathering_scan": equal,
           "device_gather_ms_untimed": round(gather_ms, 3),
           "note": "BASELINE north_star's design: windows packed with the batch (host: fc2_pack_windows from the "
                   "mmap'd FASTA; here the identical rows from fc2_gather_windows_launch), scan streams records + "
                   "reads + windows and touches no genome; whole-job throughput of this form is bound by the host "
                   "gather and PCIe (%d B/pair), so the headline keeps the resident-genome scan" % moved}
    b.win_words = b.win_nwords = None
    b.pw = 0
    torch.cuda.empty_cache()
    return out


def wave_per_pair(opt, g, b, dev, bpp, reps: int = 3):
    """North_star's kernel shape on the headline batch: one wavefront per pair (FC2_BATCH_FORM_WAVE,
    bp_wave_kernel: windows and read staged in LDS, lane = position, ballot prefix sums, wave argmax),
    timed with HIP events on the scan's stream; every result must equal the shipped form's."""
    import torch
    from find_circ2_amd import scan, _native as N
    ref = scan(opt, g, b).results[:b.n].clone()
    keep = b.layout
    b.layout = keep | N.BATCH_FORM_WAVE
    try:
        out = scan(opt, g, b)
        torch.cuda.synchronize(dev)
        equal = bool(torch.equal(out.results[:b.n], ref))
        stream = torch.cuda.current_stream(dev)
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            scan(opt, g, b, out=out)
        z.record(stream)
        torch.cuda.synchronize(dev)
        km = a.elapsed_time(z) / reps
    finally:
        b.layout = keep
    del out, ref
    ach = bpp * b.n / (km * 1e-3) / 1e9
    return {"value": round(b.n / (km * 1e-3), 1), "unit": "anchor-pairs/s", "kernel_ms": round(km, 4),
            "frac": round(ach / HBM_PEAK_GBS, 4), "results_equal_shipped_form": equal,
            "note": "BASELINE north_star's kernel shape (one wavefront per pair, 16 pairs per wave with their loads "
                    "in flight together, windows + read in LDS, lane t = positions t and t + 64, ballot/popcount "
                    "prefix sums, shuffle argmax) on the same batch and genome tables; issue-bound (DESIGN.md §4), "
                    "so the headline keeps one pair per lane"}


def cli_end_to_end(sizes=(2_000_000, 20_000_000)):
    """The product end to end (an extra, never `value`), in north_star's form ``samtools view -b ... |
    find_circ -G genome.fa -o out`` and in the metric's unit: scripts/gen_reads writes an hg19-shaped
    genome FASTA and a bwa-mem-like SAM (scripts/cli_steady.py: 60 % unspliced, 40 % spliced reads),
    fc2_sam_to_bam turns it into a BGZF BAM, and `python -m find_circ2_amd.cli` runs as its own process
    reading that BAM from a stdin pipe.  Reported per size: anchor pairs (JunctionSpans searched) per
    second of the read loop and of the process wall, and reads/s; 2M reads as the median of CLI_RUNS
    runs plus the same reads as SAM by path (files must be identical), 20M reads (steady state: the
    fixed start-up and the tables amortised) as the median of CLI_RUNS runs too (run-to-run spread on
    one box is ~10 %).  The first run builds the .byo_index."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from cli_steady import outputs, prepare, quota, run_cli
    d = tempfile.mkdtemp(prefix="fc2_bench_cli_", dir="/tmp")
    keys = ("loop_spans_per_s", "wall_spans_per_s", "loop_reads_per_s", "wall_reads_per_s", "spans", "reads",
            "loop_s", "process_wall_s", "genome_wait_s")
    try:
        small, big = min(sizes), max(sizes)
        fa, bams, sams, info = prepare(d, sizes, keep_sam_sizes=(small,))
        run_cli(fa, bams[small], os.path.join(d, "warm"), 0)
        runs = [run_cli(fa, bams[small], os.path.join(d, "bam%d" % k), 0) for k in range(CLI_RUNS)]
        order = sorted(range(len(runs)), key=lambda k: runs[k]["loop_spans_per_s"] or 0)
        med = order[len(order) // 2]
        res_small = {k: runs[med][k] for k in keys}
        res_small.update(runs_loop_spans_per_s=[r["loop_spans_per_s"] for r in runs],
                         runs_process_wall_s=[r["process_wall_s"] for r in runs], phases_s=runs[med]["phases_s"],
                         stages_s=runs[med]["stages_s"])
        by_path = run_cli(fa, sams[small], os.path.join(d, "sam_path"), 0, by_path=True)
        res_small["sam_by_path"] = {k: by_path[k] for k in keys}
        res_small["outputs_identical_bam_stdin_vs_sam_path"] = (
            outputs(os.path.join(d, "bam%d" % med)) == outputs(os.path.join(d, "sam_path")))
        big_runs = []
        for k in range(CLI_RUNS):                # (each run's files removed at once: ~2 GB at 20M reads)
            big_runs.append(run_cli(fa, bams[big], os.path.join(d, "big%d" % k), 0))
            shutil.rmtree(os.path.join(d, "big%d" % k), ignore_errors=True)
        r_big = sorted(big_runs, key=lambda r: r["loop_spans_per_s"] or 0)[len(big_runs) // 2]
        res_big = {k: r_big[k] for k in keys}
        res_big.update(runs_loop_spans_per_s=[r["loop_spans_per_s"] for r in big_runs],
                       runs_wall_spans_per_s=[r["wall_spans_per_s"] for r in big_runs],
                       phases_s=r_big["phases_s"], stages_s=r_big["stages_s"])
        return {"value": res_big["loop_spans_per_s"], "unit": "anchor-pairs/s",
                "value_process_wall": res_big["wall_spans_per_s"], "reads": big,
                "at_%dM_reads" % (small // 10**6): res_small, "at_%dM_reads" % (big // 10**6): res_big,
                "input": info, "cgroup_cpu_quota": quota(), "cpus_visible": len(os.sched_getaffinity(0)),
                "note": "whole CLI (C++ read loop + HIP search through the C context ABI), BGZF BAM piped on stdin "
                        "(cat reads.bam | python -m find_circ2_amd.cli -G genome.fa -o out), hg19-shaped genome, "
                        ".byo_index present; value = anchor pairs searched per second of the read loop at %dM reads "
                        "(value_process_wall: per second of the whole process, start-up, genome upload, BED tables "
                        "and exit included); host-bound: the loop uses the box's whole CPU share (DESIGN.md §0, "
                        "scripts/cli_steady.py for the thread curve)" % (big // 10**6)}
    except Exception as e:          # an extra must not cost the bench line
        return {"error": repr(e)}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))              # before anything touches the GPU
    import torch
    ws, rank, local = setup_dist(args)
    if ws < args.gpus:
        print("bench: --gpus %d but only %d rank(s) were started" % (args.gpus, ws), file=sys.stderr)
        sys.exit(1)
    if ws > args.gpus:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, ws), file=sys.stderr)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # wall seconds per leg of this rank (DESIGN.md §6 bounds the driver's N = 8 run from them)
    legs, t_leg = {}, [time.time()]

    def mark(name):
        now = time.time()
        legs[name] = round(now - t_leg[0], 2)
        t_leg[0] = now
    opt, g, b = build_workload(args, rank, dev)
    mark("workload")
    # the headline scan writes each pair's result as the 2-byte compact word (canonical mode; escapes
    # for results that do not fit, none on this workload): 2.2 % faster than 8-byte words in a
    # same-process A/B (profiles/r04/ab_compact_headline.jsonl), checked word for word after timing
    cw = 0 if (opt.noncanonical or opt.allhits) else HEADLINE_RESULT_BYTES
    elapsed, kernel_ms, out = timed_scans(opt, g, b, args.steps, args.warmup, ws, dev, compact_width=cw)
    elapsed = max_over_ranks(elapsed, ws, dev)
    kernel_ms = max_over_ranks(kernel_ms, ws, dev)
    mark("timed_scans")
    total_pairs = b.n * args.steps * ws
    value = total_pairs / elapsed
    bpp = algo_bytes_per_pair(args.read_len, opt.asize, opt.margin, result_bytes=cw or 8)
    achieved = bpp * b.n / (kernel_ms * 1e-3) / 1e9
    # HBM bytes per launch from the PMC passes of scripts/profile_round.sh (a --pmc pass cannot run
    # inside this process); used only for the same workload, and stamped with the commit, kernel and
    # rocprof duration it was measured on, next to this run's kernel time, so a stale value shows
    traffic, traffic_src = None, None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            w = tj.get(args.workload + ("_locus_ordered" if args.locus_ordered else ""))
            if w and int(w.get("pairs_per_launch", -1)) == b.n:
                traffic = w.get("hbm_bytes_per_launch")
                ns = w.get("avg_kernel_ns_rocprof")
                traffic_src = {"file": os.path.relpath(args.traffic_json, ROOT), "commit": w.get("commit"),
                               "kernel": w.get("kernel"), "profiled_kernel_ms": round(ns / 1e6, 4) if ns else None,
                               "this_run_kernel_ms": round(kernel_ms, 4),
                               "hbm_bytes_per_pair": w.get("hbm_bytes_per_pair")}
        except Exception:
            traffic = None
    res = out.host(b.n)
    hits = int((res["best_x"] >= 0).sum())
    b._bench_ref_results = torch.from_numpy(res.view(np.int64).copy())
    c4 = None
    if args.workload == "hg19" and not args.no_config4 and (args.config4_pairs or not args.pairs):
        c4 = configs4(opt, g, ws, rank, dev, args.steps, args.warmup, total=args.config4_pairs or 200_000_000)
        mark("configs4")
    # configs[3]: rank 0's stream strong-scaled over the ranks with the host-side ordered merge
    strong = None
    if not args.no_strong:
        n0, kw0 = workload_cfg(args, 0)
        strong = strong_scaling(opt, g, b if rank == 0 else None, b._bench_ref_results.numpy() if rank == 0 else None,
                                ws, rank, dev, args.steps, args.warmup, n0, kw0, per_rank=args.strong_batches or max(2, 8 // ws),
                                tail=args.strong_tail if args.strong_tail >= 0 else STRONG_TAIL)
        torch.cuda.empty_cache()
        mark("strong_scaling")
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "anchor-pairs/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",                 # the search's arithmetic: 32-bit integer bit planes
        "data": "synthetic (seeded; genome and anchor pairs generated on device, SURVEY.md 8(d))",
        "config": {
            "workload": ("configs[2]/[3]: hg19-shaped synthetic genome (93 @SQ contigs of test_norm.sam, 3.137 Gbp, "
                         "~7%% N) x %dM synthetic %d bp backsplice anchor pairs per GPU" % (b.n // 10**6, args.read_len))
            if args.workload == "hg19" else
            ("configs[1]: CDR1as_locus.fa x %d synthetic %d bp backsplice anchor pairs per GPU" % (b.n, args.read_len)),
            "pairs_per_gpu": b.n, "read_len": args.read_len, "asize": opt.asize, "margin": opt.margin,
            "maxdist": opt.maxdist, "parallelism": "dp%d (independent pair shards, no collective)" % ws,
            "pairs_with_hit": hits,
        },
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel_ms": round(kernel_ms, 4), "algo_bytes_per_pair": bpp,
                     "result_bytes_per_pair": cw or 8,
                     "kernel": kernel_label(g, args.locus_ordered) +
                     ("; each result written as a 2-byte compact word (fc2_bp_scan_compact_launch)" if cw else "")},
        "cpu_baseline": None,
        "strong_scaling": strong,
        "configs4_200M_150bp": c4,
    }
    if traffic:
        # HBM bytes moved per algorithmic byte (the random 19-B windows each cost whole 128-B lines)
        line["roofline"]["traffic_ratio"] = round(traffic / (bpp * b.n), 3)
    if args.workload == "hg19" and not args.locus_ordered and b.n == 50_000_000:
        pc = pattern_ceiling(opt, g, b, dev)
        mark("pattern_ceiling")
        line["roofline"]["access_pattern_ceiling"] = pc
        if pc:
            # flat copies (the driver's record keeps a line's scalar fields only): the frac this read-order
            # layout can reach at all -- the algorithmic bytes over the duration of a launch that makes
            # only the scan's memory accesses (the probe stores 8-B results, so priced with 8-B results) --
            # and how close the scan (its 8-B form, in the same run) comes to it
            bpp8 = algo_bytes_per_pair(args.read_len, opt.asize, opt.margin, result_bytes=8)
            line["roofline"]["ceiling_frac"] = round(bpp8 * b.n / (pc["probe_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            line["roofline"]["scan_frac_of_ceiling"] = pc["scan_frac_of_ceiling"]
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        cb = cpu_baselines(opt, g, b, args.cpu_seconds)
        mark("cpu_baselines")
        line["cpu_baseline"] = cb["main"]
        line["cpu_baseline_extra"] = {"python_1core": cb["python_1core"], "python_pool": cb["python_pool"],
                                      "c_naive_1core": cb["c_naive"], "c_fast_allcores": cb["c_fast"],
                                      "cpu_model": cb["cpu_model"]}
    if rank == 0 and ws == 1 and not args.no_extra and args.workload == "hg19":
        line["extra"] = {}
        if args.research:
            # the forms and pipelines DESIGN.md §5 compares the headline with (opt-in: --research)
            line["extra"]["device_pipeline_pcie"] = device_pipeline(opt, g, b, reps=5)
            line["extra"]["device_pipeline_pcie"]["d2h_8B_words"] = {
                k: v for k, v in device_pipeline(opt, g, b, reps=5, width=8).items() if k != "note"}
            line["extra"]["host_pipeline_from_pair_arrays"] = host_pipeline(opt, g, b)
            line["extra"]["configs[2]_window_carrying_batch"] = window_carrying(opt, g, b, args.steps, dev, bpp)
            line["extra"]["configs[2]_north_star_wave_per_pair_form"] = wave_per_pair(opt, g, b, dev, bpp)
            # the honest price of locus order for a read-order stream: the device reorder (fc2_reorder_launch,
            # stable counting sort by genome bucket) in front of the scan, both timed; results in input order
            line["extra"]["configs[2]_device_reorder_then_scan"] = reorder_then_scan(opt, g, b, args.steps, dev, bpp)
        del b, out
        torch.cuda.empty_cache()
        a2 = argparse.Namespace(**vars(args))
        a2.workload, a2.pairs = "cdr1as", 1_000_000
        o2, g2, b2 = build_workload(a2, rank, dev)
        el2, km2, _ = timed_scans(o2, g2, b2, max(args.steps, 20), args.warmup, 1, dev)
        line["extra"]["configs[1]_cdr1as_1M"] = {
            "value": round(b2.n * max(args.steps, 20) / el2, 1), "unit": "anchor-pairs/s",
            "kernel_ms": round(km2, 4),
            "achieved_algo_GBs": round(bpp * b2.n / (km2 * 1e-3) / 1e9, 1)}
        del b2, g2
        torch.cuda.empty_cache()
        if args.research:
            # the same configs[2] workload laid out in genome order of the A window, as
            # PairBatch.pack(locus_order=True) does on the host (results come back in input order)
            a3 = argparse.Namespace(**vars(args))
            a3.locus_ordered = True
            o3, g3, b3 = build_workload(a3, rank, dev)
            el3, km3, _ = timed_scans(o3, g3, b3, args.steps, args.warmup, 1, dev)
            ach3 = bpp * b3.n / (km3 * 1e-3) / 1e9
            line["extra"]["configs[2]_locus_ordered_batch"] = {
                "value": round(b3.n * args.steps / el3, 1), "unit": "anchor-pairs/s", "kernel_ms": round(km3, 4),
                "achieved_algo_GBs": round(ach3, 1), "frac": round(ach3 / HBM_PEAK_GBS, 4),
                "note": "same 50M-pair hg19-shaped workload, batch laid out by A-window locus (host packer option "
                        "locus_order=True); the headline keeps read order"}
            del b3, g3
            torch.cuda.empty_cache()
        # configs[4]: 200M 150 bp pairs with variable anchor lengths over 8 GPUs -> this GPU's 25M share
        a4 = argparse.Namespace(**vars(args))
        a4.pairs, a4.read_len, a4.read_len_min = 25_000_000, 150, 120
        o4, g4, b4 = build_workload(a4, rank, dev)
        bm4 = mean_algo_bytes(b4, o4.asize, o4.margin)
        el4, km4, _ = timed_scans(o4, g4, b4, args.steps, args.warmup, 1, dev)
        bpp4 = algo_bytes_per_pair(150, o4.asize, o4.margin)
        line["extra"]["configs[4]_150bp_variable_per_gpu_share"] = {
            "value": round(b4.n * args.steps / el4, 1), "unit": "anchor-pairs/s", "kernel_ms": round(km4, 4),
            "achieved_algo_GBs_at_150bp": round(bpp4 * b4.n / (km4 * 1e-3) / 1e9, 1),
            "algo_bytes_per_pair_mean": round(bm4, 2),
            "achieved_algo_GBs_at_mean": round(bm4 * b4.n / (km4 * 1e-3) / 1e9, 1),
            "note": "25M pairs (the per-GPU share of configs[4]'s 200M over 8 GPUs), read lengths uniform in "
                    "120..150 bp (anchors of varying length) and 10 %% of pair slots the two pairs of one three-segment read "
                    "(SURVEY.md 8(d) config 5), hg19-shaped genome, read order; algorithmic bytes "
                    "priced at 150 bp (%d B) and at the batch's mean read_part length" % bpp4}
        del b4, g4
        torch.cuda.empty_cache()
        mark("extras")
        if not args.no_cli:
            line["extra"]["cli_end_to_end"] = cli_end_to_end()
            mark("cli")
    if rank == 0:
        line["legs_s"] = legs
        print(json.dumps(line), flush=True)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
