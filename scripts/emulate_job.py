"""Host emulation of one STRING workgroup job (bwt.hip job_run<MODE_STRING, W>) with an exact sort:
rebuild a failing job's element set from the reference suffix array, run the job's rounds on many
input orders and report the orders whose output differs from the reference order.  Diagnostic.

    python scripts/emulate_job.py kind block_size block local_start len d [orders] [W]
"""
import importlib
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import chunkdiag  # noqa: E402

bra = importlib.import_module("br-archive_amd")
M64 = (1 << 64) - 1


class Packed:
    def __init__(self, blk: np.ndarray):
        vals = np.unique(blk)
        a = vals.size
        self.b = 1 if a <= 2 else int(a - 1).bit_length()
        rank = np.zeros(256, np.int64)
        rank[vals] = np.arange(a)
        codes = rank[blk]
        self.n = blk.size
        self.nbits = self.n * self.b
        self.nvb = (self.nbits + 7) // 8
        bits = ((codes[:, None] >> np.arange(self.b - 1, -1, -1)) & 1).astype(np.uint8).ravel()
        ext = np.concatenate([bits, bits[:512]])
        self.bits = ext

    def window(self, bp: int, nb: int) -> int:
        w = self.bits[bp: bp + nb]
        return int("".join(map(str, w.tolist())), 2) if nb else 0

    def bitpos(self, idx: int, vd: int) -> int:
        bp = idx * self.b + 8 * vd
        return bp % self.nbits if bp >= self.nbits else bp

    def load128(self, bp: int):
        sh = bp & 7
        w0 = self.window(bp, 64)
        w1 = (self.window(bp + 64, 64 - sh) << sh) if sh else self.window(bp + 64, 64)
        return w0, w1

    def load64(self, bp: int):
        sh = bp & 7
        return (self.window(bp, 64 - sh) << sh) & M64


def run_job(pk: Packed, idx_in, d: int, W: int = 2, dcap: int = 512):
    """Output rotation order (job positions) of job_run<STRING, W> for input order idx_in."""
    LOGS = {1: 8, 2: 9, 4: 10}[W]
    SM = (1 << LOGS) - 1
    ADV1 = (64 - LOGS) // 8
    ADV = (64 - 2 * LOGS) // 8
    NS = 256 * W
    T = len(idx_in)
    single = W > 1
    vd = d if single else d - 1
    Sv = [0] * NS
    Swx = [0] * NS
    key = [M64] * NS
    pos = list(range(NS))
    for c in range(NS):
        wx = 0
        v = 0
        if c < T:
            v = idx_in[c]
            w0, w1 = pk.load128(pk.bitpos(v, vd))
            key[c] = (w0 & ~SM & M64) | c
            wx = ((w0 << (8 * ADV1)) | (w1 >> (64 - 8 * ADV1))) & M64
        Sv[c] = v
        Swx[c] = wx
    order = sorted(range(NS), key=lambda c: key[c])
    key = [key[c] for c in order]
    v = [Sv[k & SM] for k in key]
    t = [Swx[k & SM] for k in key]
    key = [k & ~SM & M64 for k in key]
    Swx = t[:]
    depth = d + (ADV1 if single else ADV1 - 1)
    out = [None] * T
    Skh = [0] * NS
    rnd = 1
    while True:
        km = key
        hd = [(c == 0) or c >= T or km[c - 1] != km[c] for c in range(NS)]
        g, cur = [0] * NS, 0
        for c in range(NS):
            if hd[c]:
                cur = c
            g[c] = cur
        tied = [c < T and ((not hd[c]) or (c + 1 < T and km[c + 1] == km[c])) for c in range(NS)]
        anyt = any(tied)
        finish = not anyt
        if not finish and depth >= pk.nvb:
            finish = True
        elif not finish and depth >= dcap:
            finish = True
        T2 = 0
        if not finish:
            cx, n2 = [0] * NS, 0
            for c in range(NS):
                cx[c] = n2
                n2 += tied[c]
            T2 = n2
            nk = [0] * NS
            if rnd == 1:
                nk = [Swx[c] if tied[c] else 0 for c in range(NS)]
            Sv2 = Sv[:]
            for c in range(NS):
                if tied[c]:
                    Sv2[cx[c]] = v[c]
                    Skh[cx[c]] = ((cx[c] - (c - g[c])) << 16) | pos[c]
                    if rnd == 1:
                        Swx[cx[c]] = nk[c]
            Sv = Sv2
            key = [0] * NS
            for c in range(T2):
                key[c] = Swx[c] if rnd == 1 else pk.load64(pk.bitpos(Sv[c], depth))
        for c in range(T):
            if finish or not tied[c]:
                out[pos[c]] = v[c]
        if finish:
            break
        T = T2
        for c in range(NS):
            pos[c] = c
            if c < T:
                gp = Skh[c]
                pos[c] = gp & 0xFFFF
                key[c] = ((((gp >> 16) << (64 - LOGS)) | (key[c] >> LOGS)) & ~SM & M64) | c
            else:
                key[c] = M64
        order = sorted(range(NS), key=lambda c: key[c])
        key = [key[c] for c in order]
        v = [Sv[k & SM] for k in key]
        key = [k & ~SM & M64 for k in key]
        depth += ADV
        rnd += 1
    return out, rnd


def main():
    kind, bs, blk_i, st, ln, d = (int(x) for x in sys.argv[1:7])
    orders = int(sys.argv[7]) if len(sys.argv) > 7 else 50
    W = int(sys.argv[8]) if len(sys.argv) > 8 else 2
    blk = bra.synth_fill(kind, bs, bs, first_block=blk_i)
    sa = chunkdiag.cyclic_sa(blk)
    ref = [int(x) for x in sa[st: st + ln]]
    pk = Packed(blk)
    rng = random.Random(1)
    bad = 0
    for o in range(orders):
        inp = ref[:]
        rng.shuffle(inp)
        out, rounds = run_job(pk, inp, d, W)
        if out != ref:
            bad += 1
            wrong = [p for p in range(ln) if out[p] != ref[p]]
            print(f"order {o}: {len(wrong)} positions wrong (first {wrong[:10]}), rounds {rounds}, permutation {sorted(x for x in out if x is not None) == sorted(ref)}")
    print(f"{bad} of {orders} orders wrong (b {pk.b}, nvb {pk.nvb})")


if __name__ == "__main__":
    main()
