"""Encode one shard repeatedly; for the blocks whose digest differs from the reference, report the
first stage (BWT output, MTF output, RLE output) that differs from a round whose block matched.
GPU box diagnostic (scripts/stress_repeat.py finds the blocks)."""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from stress_repeat import D, bra, digest  # noqa: E402


def main():
    name, rank, world, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    w = D[name]
    bs, nbg = w["block_size"], w["nblocks"]
    ids = list(range(rank, nbg, world))
    codec = bra.BlockCodec(0)
    d = torch.from_numpy(bra.synth_fill(w["kind"], len(ids) * bs, bs, first_block=rank, stride=world)).cuda()
    total = d.numel()
    good, bad = {}, {}
    for r in range(rounds):
        hdr, off, pay = codec.encode(d, bs)
        torch.cuda.synchronize()
        H, O, P = hdr.cpu().numpy(), off.cpu().numpy(), pay.cpu().numpy()
        L, M = codec.stage_copy(0, total), codec.stage_copy(1, total)
        rb = codec.stage_copy(3, 8 * (len(ids) + 1)).view(np.uint64)
        rs = codec.stage_copy(4, 4 * len(ids)).view(np.uint32)
        R = codec.stage_copy(2, int(rb[len(ids)]))
        for i, g in enumerate(ids):
            ok = digest(H[i], P[O[i]:O[i + 1]].tobytes()) == w["sha256"][g]
            st = (L[i * bs:(i + 1) * bs].copy(), M[i * bs:(i + 1) * bs].copy(), R[rb[i]:rb[i] + rs[i]].copy())
            if ok and g not in good:
                good[g] = st
            if not ok:
                bad.setdefault(g, []).append((r, st))
    for g, lst in bad.items():
        for r, st in lst:
            if g not in good:
                print(f"block {g} round {r}: bad, no good round to compare", flush=True)
                continue
            gs = good[g]
            msg = []
            for nm, a, b in zip(("L", "MTF", "RLE"), st, gs):
                if a.size != b.size:
                    msg.append(f"{nm} size {a.size} vs {b.size}")
                else:
                    diff = np.flatnonzero(a != b)
                    msg.append(f"{nm} {diff.size} bytes differ (first {diff[:6].tolist()})")
            print(f"block {g} round {r}: " + "; ".join(msg), flush=True)
    print(f"rounds {rounds}, bad blocks {sorted(bad)}", flush=True)


if __name__ == "__main__":
    main()
