#!/usr/bin/env python
"""Attribute scripts/prof/sampler.c samples.  Per tag (1 = fc2_caller_next, 2 = fc2_caller_submit):
 * self: where the PC was (inlined frames of libfc2 resolved by llvm-symbolizer on a -g build;
   other objects by their dladdr symbol),
 * in-lib: the first libfc2 frame on the stack (the PC or a caller), innermost inlined function
   and its file:line -- so time in libc (memcpy, malloc) is charged to the code that called it.
usage: report.py samples.txt [top]"""
import collections
import subprocess
import sys

SYM = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def local_path(o):
    """A library of this repository named by its path on the GPU box (gpurun's scratch copy): the
    same file in this checkout, so samples taken there symbolize here."""
    import os
    i = o.find("/find_circ2_amd/")
    if i >= 0 and not os.path.exists(o):
        cand = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                            o[i + 1:])
        if os.path.exists(cand):
            return cand
    return o


def symbolize(keys):
    """{(obj, off): [(function, file:line), ...innermost first]}"""
    keys = sorted(keys)
    if not keys:
        return {}
    inp = "".join("%s 0x%x\n" % (local_path(o), off) for o, off in keys)
    out = subprocess.run([SYM, "--inlining", "--demangle", "--functions=linkage"], input=inp,
                         capture_output=True, text=True).stdout
    blocks = out.strip("\n").split("\n\n")
    res = {}
    for k, b in zip(keys, blocks):
        ls = b.splitlines()
        res[k] = [(ls[i], ls[i + 1].split("/")[-1] if i + 1 < len(ls) else "?") for i in range(0, len(ls) - 1, 2)]
    return res


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows = []
    for l in open(path):
        f = l.split()
        tag, pc, obj, base, sym = f[:5]
        callers = []
        for c in f[5:]:
            o, _, off = c.rpartition("+")
            callers.append((o, int(off, 16)))
        rows.append((tag, (obj, int(pc, 16) - int(base, 16)), sym, callers))
    lib = lambda o: "libfc2" in o.split("/")[-1]      # noqa: E731
    keys = set()
    for _, pc, _, callers in rows:
        for o, off in [pc] + callers:
            if lib(o):
                keys.add((o, off if (o, off) == pc else off - 1))
    names = symbolize(keys)
    for tag in sorted({r[0] for r in rows}):
        sel = [r for r in rows if r[0] == tag]
        selfc, inlib, inlib_outer, inlib_line, own_line = (collections.Counter() for _ in range(5))
        for _, pc, sym, callers in sel:
            if lib(pc[0]):
                fr = names.get(pc, [("?", "?")])
                selfc[fr[0][0][:100]] += 1
            else:
                selfc["%s:%s" % (pc[0].split("/")[-1], sym)] += 1
            chain = [pc] + [(o, off - 1) for o, off in callers]
            first = next(((o, off) for o, off in chain if lib(o)), None)
            if first is None:
                inlib["(outside libfc2)"] += 1
                continue
            fr = names.get(first, [("?", "?")])
            inlib[fr[0][0][:100]] += 1
            inlib_outer[fr[-1][0][:100]] += 1
            inlib_line[fr[0][1]] += 1
            own = next((f for f in fr if f[1].startswith("fc2_")), None)    # the innermost line of our sources
            own_line["%s  %s" % (own[1], own[0][:60]) if own else "?"] += 1
        n = len(sel)
        print("== tag %s: %d samples" % (tag, n))
        for title, c in (("self", selfc), ("in-lib (innermost)", inlib), ("in-lib (outermost)", inlib_outer),
                         ("in-lib line", inlib_line), ("own source line", own_line)):
            print("-- %s" % title)
            for k, v in c.most_common(top):
                print("%6.1f%%  %s" % (100.0 * v / n, k))


if __name__ == "__main__":
    main()
