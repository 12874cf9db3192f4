"""Random-gather micro-benchmark driver (measurement only): python scripts/micro/gather.py [modes...]
Prints one JSON line per mode: ms per launch and gathers per ns.  See gather.hip for the modes."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libgather.so"))
SBYTES = 224 << 20
N = 64 << 20  # gathers per launch
g = torch.Generator(device="cpu").manual_seed(1)
s = torch.randint(0, 256, (SBYTES + 64,), dtype=torch.uint8, generator=g).cuda()
idx = torch.randint(0, SBYTES - 32, (N,), dtype=torch.int64, generator=g).to(torch.int32).cuda()
out = torch.empty(N // 4, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
ms = ctypes.c_float()
for m in [int(x) for x in sys.argv[1:]] or range(7):
    rc = lib.gather_run(ctypes.c_void_p(s.data_ptr()), ctypes.c_void_p(idx.data_ptr()), ctypes.c_uint64(N), m,
                        ctypes.c_void_p(out.data_ptr()), 10, ctypes.byref(ms))
    assert rc == 0, rc
    print(json.dumps({"mode": m, "ms": round(ms.value, 4), "gathers_per_ns": round(N / ms.value / 1e6, 2)}), flush=True)
