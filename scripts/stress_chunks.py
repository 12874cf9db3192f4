"""Repeat the 1024 x 256 KiB chunk-stream round trip in one process, each round preceded by
smaller encodes/decodes of other geometries on the same codec (the order of tests/test_gpu_chunks.py),
and localise every failure: chunk records vs the reference digests, then the decode per chunk and
stage (tests/chunkdiag.py).  Prints one line per round; exits 1 on any mismatch.  GPU diagnostic.

    python scripts/stress_chunks.py [rounds]
"""
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import chunkdiag  # noqa: E402
from oracle import Oracle  # noqa: E402

bra = importlib.import_module("br-archive_amd")
CS = 256 * 1024


def prelude(codec, r):
    """Other geometries first: small chunk streams and a 1 MiB-block batch (as the test module)."""
    for kind, total, bs in [(0, 8 << 20, 1 << 20), (2, 3 * CS + 1, CS), (1, 2 * CS, CS), (0, 1, CS), (0, 6 * CS + 77, CS)][: 1 + r % 5]:
        d = torch.from_numpy(bra.synth_fill(kind, total, bs)).cuda()
        st, _, comp = codec.compress_chunks(d, bs)
        if comp and bs == CS:
            out, _ = codec.decompress_chunks(st, bs)
            assert torch.equal(out, d), ("prelude", kind, total)


def one(codec, orc, D, name):
    w = D[name]
    bs, nb = w["block_size"], w["nblocks"]
    total = bs * nb
    data = bra.synth_fill(w["kind"], total, bs)
    d = torch.from_numpy(data).cuda()
    stream, crc, compressed = codec.compress_chunks(d, CS)
    st = stream.cpu().numpy().tobytes()
    bad = chunkdiag.records_vs_reference(st, w)
    if bad:
        return f"ENCODE {len(bad)} records differ, first {bad[:8]}; " + "; ".join(
            chunkdiag.encode_diagnosis(codec, orc, data, b, bs, total, st) for b in bad[:3])
    want = orc.chunks_crc32c(chunkdiag.headers_in_memory(st), data.tobytes(), CS)
    if crc != want:
        return f"ENCODE crc {crc:#x} != {want:#x}"
    if not compressed:
        return "ok (stored)"
    out, dcrc = codec.decompress_chunks(stream, CS, out_cap=total)
    bad = chunkdiag.bad_chunks(out.cpu().numpy(), data, bs)
    if bad:
        first = bad[0] if bad[0] >= 0 else 0
        return f"DECODE {len(bad)} chunks differ, first {bad[:8]}; {chunkdiag.decode_diagnosis(codec, orc, data, first, bs, total)}"
    if dcrc != crc:
        return f"DECODE crc {dcrc:#x} != {crc:#x}"
    return "ok"


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    pre = int(sys.argv[2]) if len(sys.argv) > 2 else -1  # fixed prelude (-1: rotate through them)
    codec = bra.BlockCodec(0)
    orc = Oracle()
    D = chunkdiag.load_digests()
    fails = 0
    for r in range(rounds):
        t0 = time.time()
        prelude(codec, r if pre < 0 else pre)
        res = {n: one(codec, orc, D, n) for n in ("text_256KiB_x1024", "sym16_256KiB_x1024")}
        fails += sum(not v.startswith("ok") for v in res.values())
        print(f"round {r}: {time.time() - t0:.1f} s {res}", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
