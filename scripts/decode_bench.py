"""Decode alone (measurement tooling): encode 256 MiB of synthetic blocks once, then time the
device decode and its stages, and check the round trip.  The library is BRA_HIP_LIB's (A/B of
measurement variants) or the in-tree one.

    python scripts/decode_bench.py [kind] [block_size] [reps]      -> one JSON line
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench

    kind = sys.argv[1] if len(sys.argv) > 1 else "text"
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    bra = importlib.import_module("br-archive_amd")
    total = 256 << 20
    d = torch.from_numpy(bra.synth_fill(bench.KINDS[kind], total, bs)).cuda()
    codec = bra.BlockCodec(0)
    H, O, P = codec.encode(d, bs)
    out = codec.decode(H, O, P, total, bs)  # warm-up (allocations)
    torch.cuda.synchronize()
    ok = bool(torch.equal(out, d))
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.decode(H, O, P, total, bs, out=out)
    torch.cuda.synchronize()
    gbps = reps * total / (time.perf_counter() - t0) / 1e9
    ok = ok and bool(torch.equal(out, d))
    slots = [s for s in codec.SLOTS if s.startswith("dec.")]
    codec.prof_enable(codec.slot_mask(*slots))
    codec.prof_reset()
    codec.decode(H, O, P, total, bs, out=out)
    torch.cuda.synchronize()
    dp = codec.prof_read()
    codec.prof_enable(0)
    print(json.dumps({"kind": kind, "block_size": bs, "decode_GBps": round(gbps, 3), "roundtrip_ok": ok,
                      "ms": {s: round(dp[s][0] / max(1, dp[s][1]), 4) for s in slots if s in dp}}), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
