"""Experiment: consecutive encode steps of the bench workload alternating over P contexts / streams
(step k on context k % P), so that step k's MTF / RLE / Huffman tail overlaps step k + 1's BWT.
Prints ms per step and GB/s for each P; checks that every context's headers match.
    python scripts/exp_pipeline.py [P ...]"""
import importlib
import json
import sys
import time

import torch

sys.path.insert(0, ".")
bra = importlib.import_module("br-archive_amd")
bs, total, steps = 1 << 20, 256 << 20, 12
d = torch.from_numpy(bra.synth_fill(0, total, bs)).cuda()
nb = total // bs
ref = None
for P in [int(x) for x in sys.argv[1:]] or [1, 2]:
    codecs = [bra.BlockCodec(0) for _ in range(P)]
    streams = [torch.cuda.Stream() for _ in range(P)]
    bufs = [(torch.empty((nb, 268), dtype=torch.uint8, device="cuda"), torch.empty((nb + 1,), dtype=torch.int64, device="cuda"),
             torch.empty((int(total * 1.25) + 64 * nb + 65536,), dtype=torch.uint8, device="cuda")) for _ in range(P)]
    crc = [torch.zeros((1,), dtype=torch.int32, device="cuda") for _ in range(P)]

    def step(k):
        c = k % P
        with torch.cuda.stream(streams[c]):
            h, o, p = bufs[c]
            codecs[c].encode(d, bs, h, o, p, stream=streams[c])
            codecs[c].chunks_crc32c_shard(d, h, bs, 0, 1, total, True, out=crc[c], stream=streams[c])

    for k in range(2 * P):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    hs = [b[0].cpu() for b in bufs]
    same = all(torch.equal(hs[0], h) for h in hs) and (ref is None or torch.equal(ref, hs[0]))
    ref = hs[0] if ref is None else ref
    print(json.dumps({"contexts": P, "ms_per_step": round(el * 1e3, 3), "GBps": round(total / el / 1e9, 3), "headers_equal": same}), flush=True)
    for c in codecs:
        c.close()
