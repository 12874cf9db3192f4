"""Experiment: the batch split over K contexts, each driven by its own host thread on its own stream
(independent stages of different sub-batches overlap on the device).  usage: exp_streams.py [K ...]"""
import importlib
import sys
import threading
import time

import torch

sys.path.insert(0, ".")
from bench import KINDS  # noqa: E402

bra = importlib.import_module("br-archive_amd")
bs, total = 1 << 20, 256 << 20
kind = KINDS[sys.argv[1]] if len(sys.argv) > 1 and sys.argv[1] in KINDS else KINDS["text"]
ks = [int(x) for x in sys.argv[1:] if x.isdigit()] or [1, 2, 4]
d = torch.from_numpy(bra.synth_fill(kind, total, bs)).cuda()
ref = None
for K in ks:
    per = total // K
    codecs = [bra.BlockCodec(0) for _ in range(K)]
    streams = [torch.cuda.Stream() for _ in range(K)]
    outs = [None] * K

    def run(i):
        with torch.cuda.stream(streams[i]):
            outs[i] = codecs[i].encode(d[i * per:(i + 1) * per], bs, stream=streams[i])
            streams[i].synchronize()

    def loop(i, n, delay):
        time.sleep(delay * i)
        for _ in range(n):
            run(i)

    def step():
        th = [threading.Thread(target=run, args=(i,)) for i in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / n
    hdr = torch.cat([o[0] for o in outs]).cpu()
    same = ref is None or torch.equal(hdr, ref)
    ref = hdr if ref is None else ref
    # staggered: each context encodes its sub-batch 8 times, context i starting i * (step / K / 2) later
    t0 = time.perf_counter()
    th = [threading.Thread(target=loop, args=(i, 8, el / K / 2)) for i in range(K)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    el2 = (time.perf_counter() - t0) / 8
    print(f"K={K} staggered: {el2 * 1e3:.2f} ms per full batch {total / el2 / 1e9:.2f} GB/s", flush=True)
    print(f"K={K}: {el * 1e3:.2f} ms/step {total / el / 1e9:.2f} GB/s headers_equal={same}", flush=True)
