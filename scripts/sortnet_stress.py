"""Stress the job sort (bitonic network in registers + merge levels) alone on the GPU:
bra_gpu_sortnet_selftest(waves, groups, iters, seed, keys) sorts groups x iters key sets per call
(random ones, or the 256 * waves keys of a sort_dump.bin of the job audit) and returns the failing
count.  GPU diagnostic.

    python scripts/sortnet_stress.py [reps] [lib path] [sort_dump.bin]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
path = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-" else os.path.join(ROOT, "br-archive_amd", "libbra_hip.so")
dump = sys.argv[3] if len(sys.argv) > 3 else None
lib = C.CDLL(path)
f = lib.bra_gpu_sortnet_selftest
f.argtypes = [C.c_int, C.c_uint, C.c_uint, C.c_uint, C.c_void_p]
f.restype = C.c_int
res = {}
if dump:
    raw = open(dump, "rb").read()
    meta = np.frombuffer(raw[:16], np.uint32)
    keys = np.ascontiguousarray(np.frombuffer(raw[16:], np.uint64).reshape(2, 1024)[0])
    w = int(meta[0])
    tot = 0
    for r in range(reps):
        tot += f(w, 1024, 16, r, C.c_void_p(keys.ctypes.data))
    res[w] = {"sorts": reps * 1024 * 16, "failed": tot, "keys": os.path.basename(dump)}
else:
    for w in (1, 2, 4):
        tot, t0 = 0, time.time()
        for r in range(reps):
            e = f(w, 8192 // w, 64, 1000 * w + r, None)
            if e < 0:
                print(json.dumps({"error": "launch", "waves": w}))
                sys.exit(2)
            tot += e
        res[w] = {"sorts": reps * (8192 // w) * 64, "failed": tot, "s": round(time.time() - t0, 2)}
print(json.dumps({"lib": os.path.relpath(path, ROOT), "results": res}), flush=True)
sys.exit(1 if any(v["failed"] for v in res.values()) else 0)
