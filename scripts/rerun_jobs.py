"""Encode a workload once, then re-run its BWT job phase many times on the unchanged job lists and
payloads, auditing every run (needs a -DBRA_JOB_AUDIT build in BRA_HIP_LIB).  Prints the failing
jobs per batch of re-runs.  GPU diagnostic.

    BRA_HIP_LIB=.../audit/libbra_hip.so python scripts/rerun_jobs.py [kind] [block_size] [nblocks] [reps] [shuffle seed]
"""
import ctypes as C
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bra = importlib.import_module("br-archive_amd")

kind = int(sys.argv[1]) if len(sys.argv) > 1 else 0
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 256 * 1024
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 200
seed = int(sys.argv[5]) if len(sys.argv) > 5 else 0
f = bra.lib.bra_gpu_debug_rerun_jobs
f.argtypes = [C.c_void_p, C.c_int, C.c_uint]
f.restype = C.c_int
codec = bra.BlockCodec(0)
d = torch.from_numpy(bra.synth_fill(kind, bs * nb, bs)).cuda()
codec.encode(d, bs)
torch.cuda.synchronize()
out = []
t0 = time.time()
for i in range(0, reps, 20):
    r = f(codec.ctx, min(20, reps - i), (seed + i) if seed else 0)
    out.append(r)
    print(json.dumps({"batch": i // 20, "failing_jobs": r, "s": round(time.time() - t0, 1)}), flush=True)
    if r < 0:
        sys.exit(2)
print(json.dumps({"kind": kind, "block_size": bs, "nblocks": nb, "reps": reps, "failing_jobs": sum(out)}))
