"""HIP initialisation time of the CLI's first context (fc2_ctx_create on a fresh process) under a few
runtime settings, 5 runs each, one JSON line per setting: the first HIP call's cost is the longest
fixed item of the CLI's start-up (DESIGN.md §5 "Start-up")."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import ctypes, sys, time, json
t0 = time.time()
L = ctypes.CDLL(%r)
t1 = time.time()
L.fc2_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
c = ctypes.c_void_p()
rc = L.fc2_ctx_create(0, ctypes.byref(c))
t2 = time.time()
print(json.dumps({"dlopen_s": round(t1 - t0, 4), "ctx_create_s": round(t2 - t1, 4), "rc": rc}))
import os; os._exit(0)
"""
SETTINGS = [{}, {"HIP_ENABLE_DEFERRED_LOADING": "0"}, {"HIP_ENABLE_DEFERRED_LOADING": "1"},
            {"GPU_MAX_HW_QUEUES": "1"}, {"HSA_ENABLE_SDMA": "0"}, {"AMD_SERIALIZE_KERNEL": "0"},
            {"HIP_VISIBLE_DEVICES": "0"}, {"ROCR_VISIBLE_DEVICES": "0"}]


def main():
    lib = os.path.join(ROOT, "find_circ2_amd", "libfc2.so")
    for extra in SETTINGS:
        env = dict(os.environ, **extra)
        runs = []
        for _ in range(5):
            r = subprocess.run([sys.executable, "-c", CHILD % lib], env=env, stdout=subprocess.PIPE, timeout=120)
            runs.append(json.loads(r.stdout.decode().strip().splitlines()[-1]))
        cc = sorted(x["ctx_create_s"] for x in runs)
        print(json.dumps({"env": extra, "ctx_create_s": cc, "median": cc[2],
                          "dlopen_s": sorted(x["dlopen_s"] for x in runs)[2]}), flush=True)


if __name__ == "__main__":
    main()
