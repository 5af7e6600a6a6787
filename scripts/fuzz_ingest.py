#!/usr/bin/env python
"""Damaged-input campaign over the readers (the seeded cases of tests/test_ingest_fuzz.py, many more
of them).  Run it against a sanitizer build of the host code, as scripts/sanitize_host.sh builds one:

    FC2_LIB_VARIANT=asan LD_PRELOAD=<clang asan runtime> ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 \\
        python scripts/fuzz_ingest.py ingest|cli|python SEED0 N

ingest: the native reader (fc2_ingest_next) to the end of each case; cli: the whole CLI with the
native read loop, -B, and the CPU oracle as evaluator; python: the --python-ingest reader, which must
raise only OSError / ValueError.  Prints the outcome counts; a memory error aborts the run."""
import collections
import gzip
import os
import random
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

from samgen import bgzf_compress, sam_to_bam  # noqa: E402
from test_ingest import _mixed_sam  # noqa: E402
from test_ingest_fuzz import _damage, _native_all, _python_all  # noqa: E402


def main():
    mode, seed0, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    d = tempfile.mkdtemp()
    sam = os.path.join(d, "m.sam")
    fa = _mixed_sam(sam, 160, seed=815)
    text = open(sam, "rb").read()
    data = {"sam": text, "sam_bgzf": bgzf_compress(text), "sam_gzip": gzip.compress(text)}
    for form, comp in (("bam_bgzf", "bgzf"), ("bam_gzip", "gzip"), ("bam_raw", "none")):
        p = os.path.join(d, form)
        sam_to_bam(text.decode("latin-1"), p, compress=comp)
        data[form] = open(p, "rb").read()
    out = collections.Counter()
    for s in range(seed0, seed0 + n):
        rng = random.Random(s)
        form = sorted(data)[s % len(data)]
        p = os.path.join(d, "case")
        with open(p, "wb") as fh:
            fh.write(_damage(rng, data[form]))
        try:
            if mode == "ingest":
                _native_all(p)
                out["ok"] += 1
            elif mode == "python":
                _python_all(p)
                out["ok"] += 1
            else:
                from find_circ2_amd import cli
                from oracle_engine import oracle_evaluator_factory
                rc = cli.main(["-G", fa, "-o", os.path.join(d, "o"), "-q", "-B", p],
                              evaluator_factory=oracle_evaluator_factory)
                out["exit %d" % rc] += 1
        except (OSError, ValueError, RuntimeError) as ex:
            out["error " + type(ex).__name__] += 1
    print(mode, seed0, n, dict(out), flush=True)


if __name__ == "__main__":
    main()
