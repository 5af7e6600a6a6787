#!/usr/bin/env python
"""Damaged-genome campaign (the seeded cases of tests/test_fasta_fuzz.py, many more of them): FASTA
text cut / flipped / spliced, and .byo_index fields set to nonsense, through fc2_fasta_open, layout,
pack and random windows.  Run it against a sanitizer build as scripts/fuzz_ingest.py says:

    FC2_LIB_VARIANT=asan LD_PRELOAD=<clang asan runtime> python scripts/fuzz_fasta.py SEED0 N
"""
import ctypes, os, sys, random, tempfile, collections
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from find_circ2_amd import _native as N
L = N.lib()
gold = [open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", f), "rb").read() for f in ("CDR1as_locus.fa", "test_ref.fa")]
d = tempfile.mkdtemp()
def damage_fa(rng, b):
    b = bytearray(b); k = rng.randrange(5)
    if k == 0: return bytes(b[:rng.randrange(len(b) + 1)])
    if k == 1:
        for _ in range(rng.randint(1, 6)):
            i = rng.randrange(len(b)); b[i] = rng.choice(b"ACGTNacgtn>\r\n \tRYK#\x00\xff")
        return bytes(b)
    if k == 2:
        i = rng.randrange(len(b)); return bytes(b[:i]) + bytes(rng.randrange(256) for _ in range(rng.randint(1, 40))) + bytes(b[i:])
    if k == 3:   # line lengths changed
        lines = bytes(b).split(b"\n"); i = rng.randrange(len(lines)); lines[i] = lines[i][:rng.randrange(len(lines[i]) + 1)]
        return b"\n".join(lines)
    return bytes(rng.randrange(256) for _ in range(rng.randint(0, 200)))
def damage_idx(rng, text):
    lines = text.split(b"\n"); i = rng.randrange(len(lines)); parts = lines[i].split(b"\t")
    if len(parts) == 6:
        j = rng.randrange(6)
        parts[j] = rng.choice([b"-5", b"0", b"999999999", b"-999999999999", b"9223372036854775807", b"'\\x'", b"'", b"x", b""])
        lines[i] = b"\t".join(parts)
    return b"\n".join(lines)
out = collections.Counter()
for s in range(int(sys.argv[1]), int(sys.argv[1]) + int(sys.argv[2])):
    rng = random.Random(s)
    fa = os.path.join(d, "g%d.fa" % (s % 3))
    for ext in ("", ".byo_index"):
        try: os.unlink(fa + ext)
        except FileNotFoundError: pass
    src = gold[s % 2]
    use_idx = rng.random() < 0.5
    data = src if use_idx else damage_fa(rng, src)
    open(fa, "wb").write(data)
    h = ctypes.c_void_p()
    if use_idx:
        rc = L.fc2_fasta_open(fa.encode(), 1, ctypes.byref(h))
        if rc == 0: L.fc2_fasta_close(h)
        if os.path.exists(fa + ".byo_index"):
            t = open(fa + ".byo_index", "rb").read(); os.chmod(fa + ".byo_index", 0o644)
            open(fa + ".byo_index", "wb").write(damage_idx(rng, t))
    rc = L.fc2_fasta_open(fa.encode(), 0, ctypes.byref(h))
    if rc != 0: out["open_err"] += 1; continue
    try:
        nu, ncw = ctypes.c_uint64(), ctypes.c_uint64()
        nch = L.fc2_fasta_n_chrom(h)
        cs = np.zeros(max(1, nch), np.uint64)
        if L.fc2_fasta_layout(h, ctypes.byref(nu), ctypes.byref(ncw), cs.ctypes.data) != 0: out["layout_err"] += 1; continue
        if nu.value > 50_000_000: out["huge"] += 1; continue
        units = np.empty(2 * nu.value, np.uint64); npl = np.empty(nu.value, np.uint64); nc = np.zeros(max(1, ncw.value), np.uint32)
        ne = ctypes.c_uint64()
        rc = L.fc2_fasta_pack(h, units.ctypes.data, npl.ctypes.data, nc.ctypes.data, ctypes.byref(ne), 2)
        out["pack_ok" if rc == 0 else "pack_err"] += 1
        buf = np.zeros(4096, np.uint8); ln = ctypes.c_int64()
        for _ in range(20):
            c = rng.randrange(-1, nch + 1); a = rng.randrange(-3000, 5000); b = a + rng.randrange(-10, 300)
            L.fc2_fasta_get_upper(h, c, a, b, buf.ctypes.data, 4096, ctypes.byref(ln))
    finally:
        L.fc2_fasta_close(h)
print(dict(out))
