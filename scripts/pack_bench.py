"""Host pair packer throughput (fc2_pack_pairs) on this machine: 100 bp read parts, ACGT with
0.05 % 'N', 4M pairs, 1..16 threads, best of 5.  Prints one JSON line per thread count."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from find_circ2_amd import _native as N  # noqa: E402

n, L = 4_000_000, 100
rng = np.random.default_rng(1)
buf = rng.choice(np.frombuffer(b"ACGT", np.uint8), n * L + 16)
buf[rng.random(n * L + 16) < 0.0005] = ord("N")
off = np.arange(n, dtype=np.uint64) * np.uint64(L)
hp = np.zeros(n, N.PAIR_DTYPE)
hp["a_pos"] = rng.integers(0, 2000, n)
hp["b_aend"] = hp["a_pos"] + 300
hp["read_len"] = L
p = N.Params(15, 2, 2, 0, 0, 0, 0)
words = np.zeros(3 * n, np.uint64)
nwords = np.zeros(2 * n, np.uint64)
nbp = ctypes.c_uint64()
for T in [int(a) for a in (sys.argv[1:] or ["1", "4", "8", "16"])]:
    best = 1e9
    for _ in range(5):
        t = time.perf_counter()
        N.check(N.lib().fc2_pack_pairs(ctypes.byref(p), None, n, buf.ctypes.data, off.ctypes.data, hp.ctypes.data,
                                       words.ctypes.data, 3, nwords.ctypes.data, 2, n, ctypes.byref(nbp), T))
        best = min(best, time.perf_counter() - t)
    print(json.dumps({"threads": T, "ns_per_pair": round(best / n * 1e9, 2), "pairs_per_s": round(n / best, 1)}),
          flush=True)
