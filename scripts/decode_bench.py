"""Decode throughput of the batch API (output GB/s), one workload: encode once, decode R times."""
import argparse
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

KINDS = {"text": 0, "random": 1, "sym16": 2, "tiled": 3}
ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="text")
ap.add_argument("--block-size", type=int, default=1 << 20)
ap.add_argument("--total", type=int, default=256 << 20)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
bra = importlib.import_module("br-archive_amd")
data = bra.synth_fill(KINDS[args.kind], args.total, args.block_size)
d = torch.from_numpy(data).cuda()
codec = bra.BlockCodec(0)
hdr, off, pay = codec.encode(d, args.block_size)
out = codec.decode(hdr, off, pay, args.total, args.block_size)
torch.cuda.synchronize()
ok = bool(torch.equal(out, d))
t0 = time.perf_counter()
for _ in range(args.reps):
    codec.decode(hdr, off, pay, args.total, args.block_size, out=out)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / args.reps
# one more decode with the decode slots timed
codec.prof_enable(codec.slot_mask("dec.huffman", "dec.rle", "dec.mtf", "dec.ibwt", *codec.DECODE_KERNELS))
codec.prof_reset()
codec.decode(hdr, off, pay, args.total, args.block_size, out=out)
torch.cuda.synchronize()
prof = {k: round(v[0], 3) for k, v in codec.prof_read().items() if v[1]}
codec.prof_enable(0)
print(json.dumps({"kind": args.kind, "block_size": args.block_size, "decode_GBps": round(args.total / dt / 1e9, 4), "ms": round(dt * 1e3, 3),
                  "roundtrip": ok, "lib": os.path.basename(os.path.dirname(bra.LIB_PATH)), "slots_ms": prof}))
