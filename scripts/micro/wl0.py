"""Wide level-0 scatter micro-benchmark driver (measurement only): python scripts/micro/wl0.py [P ...]
Builds libwl0.so from wl0.hip if needed; one JSON line per part count P: ms per launch over
256 x 1 MiB synthetic text, and whether every slot was written exactly once."""
import ctypes
import importlib
import json
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
bra = importlib.import_module("br-archive_amd")
so = os.path.join(HERE, "libwl0.so")
if not os.path.exists(so):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so, os.path.join(HERE, "wl0.hip")])
lib = ctypes.CDLL(so)
lib.wl0_launch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint32] * 2 + [ctypes.c_void_p] * 3 + [ctypes.c_uint32, ctypes.c_void_p]
n, nb = 1 << 20, int(os.environ.get("NB", "256"))
kind = int(os.environ.get("KIND", bra.SYNTH_TEXT))
h = bra.synth_fill(kind, n * nb, n)
vals = np.unique(h)
assert len(vals) <= 32, len(vals)
rank = np.zeros(256, np.uint8)
rank[vals] = np.arange(len(vals))
d = torch.from_numpy(h).cuda()
rk = torch.from_numpy(rank).cuda()
c = rk[d.long()].view(nb, n).long()
cs = [torch.roll(c, -k, dims=1) for k in range(4)]
d16 = (cs[0] << 11) | (cs[1] << 6) | (cs[2] << 1) | (cs[3] >> 4)
cnt = torch.bincount((d16 + torch.arange(nb, device="cuda").view(nb, 1) * 65536).view(-1), minlength=nb * 65536).view(nb, 65536)
starts = (torch.cumsum(cnt, 1) - cnt + torch.arange(nb, device="cuda").view(nb, 1) * n).to(torch.int32).contiguous()
del cs, c, cnt
opay = torch.empty(n * nb, dtype=torch.int64, device="cuda")
odig = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
lib.wl0_set_attr()
s = torch.cuda.current_stream().cuda_stream
for P in [int(a) for a in sys.argv[1:]] or [2, 4, 8, 16]:
    def run():
        assert lib.wl0_launch(d.data_ptr(), rk.data_ptr(), n, nb, starts.data_ptr(), opay.data_ptr(), odig.data_ptr(), P, s) == 0
    opay.fill_(-1)
    run()
    torch.cuda.synchronize()
    idx = (opay & 0xFFFFF).view(nb, n)
    ok = bool((opay != -1).all()) and bool((torch.sort(idx, dim=1).values == torch.arange(n, device="cuda")).all())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        run()
    ev[0].record()
    reps = 10
    for _ in range(reps):
        run()
    ev[1].record()
    torch.cuda.synchronize()
    print(json.dumps({"P": P, "ms": ev[0].elapsed_time(ev[1]) / reps, "exact_once": ok, "blocks": nb, "kind": kind}), flush=True)
