"""Stress helper: repeat encodes of several workloads in one process and compare the BWT (L + pi)
of chosen blocks with the oracle every time (hunts non-deterministic BWT results)."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from oracle import Oracle

bra = importlib.import_module("br-archive_amd")
orc = Oracle()
codec = bra.BlockCodec(0)
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
work = [(0, 1 << 20, 256, [0, 77]), (2, 65536, 64, [0, 5]), (1, 1 << 20, 256, [0]), (2, 8 << 20, 4, [0, 1, 2, 3]), (3, 1 << 20, 16, [0])]
refs = {}
datas = {}
for kind, bs, nb, chk in work:
    data = bra.synth_fill(kind, bs * nb, bs)
    datas[(kind, bs)] = torch.from_numpy(data).cuda()
    for b in chk:
        L, pi = orc.bwt_encode(data[b * bs:(b + 1) * bs].tobytes())
        refs[(kind, bs, b)] = (np.frombuffer(L, np.uint8), pi)
bad = 0
for it in range(iters):
    for kind, bs, nb, chk in work:
        hdr, off, pay = codec.encode(datas[(kind, bs)], bs)
        L = codec.stage_copy(0, bs * nb)
        hdr_h = hdr.cpu().numpy()
        for b in chk:
            rL, rpi = refs[(kind, bs, b)]
            pi = bra.parse_header(hdr_h[b].tobytes())[0]
            nbad = int((L[b * bs:(b + 1) * bs] != rL).sum())
            if pi != rpi or nbad:
                bad += 1
                print(f"iter {it} kind {kind} bs {bs} block {b}: pi {pi} ref {rpi}; L mismatches {nbad}", flush=True)
    print(f"iter {it} done, bad so far {bad}", flush=True)
sys.exit(1 if bad else 0)
