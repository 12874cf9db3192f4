"""Host statistics of the BWT job phase (bwt.hip job_run) on a synthetic block: the MSD buckets that
become jobs (<= 1024 elements, split on packed key bytes like the device levels), and for each job
the distribution of its next key byte -- what an in-job counting pass on that byte would leave for
the sort networks.  Measurement / design aid only (CPU, numpy).

    python scripts/job_bins.py [kind] [block_size] [blocks]
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bra = importlib.import_module("br-archive_amd")

NB = 20  # packed key bytes kept per rotation (deeper buckets are counted as jobs at that depth)


def packed_bytes(blk: np.ndarray) -> np.ndarray:
    vals = np.unique(blk)
    b = 1 if vals.size <= 2 else int(vals.size - 1).bit_length()
    rank = np.zeros(256, np.int64)
    rank[vals] = np.arange(vals.size)
    codes = rank[blk]
    n = blk.size
    bits = ((codes[:, None] >> np.arange(b - 1, -1, -1)) & 1).astype(np.uint8).ravel()
    ext = np.concatenate([bits, bits[: NB * 8 + 64]])
    # rotation i starts at bit i*b; take NB bytes
    starts = np.arange(n) * b
    out = np.zeros((n, NB), np.uint8)
    for j in range(NB * 8):
        out[:, j // 8] |= (ext[starts + j] << (7 - (j & 7))).astype(np.uint8)
    return out, b


def jobs_of(keys: np.ndarray, order: np.ndarray):
    """(start, end, depth) of every job: buckets of <= 1024 rotations after the MSD levels."""
    out = []
    stack = [(0, keys.shape[0], 0)]
    k = keys[order]
    while stack:
        s, e, d = stack.pop()
        if d >= NB:
            out.append((s, e, d))
            continue
        col = k[s:e, d]
        # sub-buckets of byte d (sorted, so contiguous)
        cuts = np.flatnonzero(np.diff(col.astype(np.int16))) + 1
        bounds = np.concatenate([[0], cuts, [e - s]])
        for a, z in zip(bounds[:-1], bounds[1:]):
            if z - a <= 1:
                continue  # a single rotation is placed by the scan
            if z - a <= 1024:
                out.append((s + a, s + z, d + 1))
            else:
                stack.append((s + a, s + z, d + 1))
    return out, k


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "text"
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    nblk = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    kid = {"text": bra.SYNTH_TEXT, "random": bra.SYNTH_RANDOM, "sym16": bra.SYNTH_SYM16}[kind]
    data = bra.synth_fill(kid, bs * nblk, bs)
    stats = {"wave": [], "wg2": [], "wg4": []}
    for bi in range(nblk):
        blk = data[bi * bs:(bi + 1) * bs]
        keys, b = packed_bytes(blk)
        order = np.lexsort(keys.T[::-1])
        jobs, k = jobs_of(keys, order)
        for s, e, d in jobs:
            n = e - s
            cls = "wave" if n <= 256 else ("wg2" if n <= 512 else "wg4")
            if d >= NB:
                continue
            dig = k[s:e, d]
            cnt = np.bincount(dig, minlength=256)
            cnt = cnt[cnt > 0]
            # 12-bit digit: byte d and the high nibble of byte d+1
            d12 = (dig.astype(np.int32) << 4) | (k[s:e, d + 1] >> 4 if d + 1 < NB else 0)
            c12 = np.bincount(d12)
            c12 = c12[c12 > 0]
            stats[cls].append((n, cnt.max(), (cnt == 1).sum(), cnt.size, (cnt ** 2).sum(), c12.max(), (c12 ** 2).sum()))
    for cls, v in stats.items():
        if not v:
            continue
        a = np.array(v, np.float64)
        n = a[:, 0]
        p2 = lambda x: 2 ** np.ceil(np.log2(np.maximum(x, 2)))  # noqa: E731
        print(f"{kind} {cls}: jobs {len(v)} elements {int(n.sum())} mean len {n.mean():.0f}; "
              f"8-bit digit: max bin mean {a[:, 1].mean():.1f} (p50 {np.median(a[:, 1]):.0f}, p90 {np.percentile(a[:, 1], 90):.0f}), "
              f"singletons {a[:, 2].sum() / n.sum():.1%}, bins {a[:, 3].mean():.1f}, sum sq / n {a[:, 4].sum() / n.sum():.1f}; "
              f"network size of max bin / job network: {(p2(a[:, 1]) * n).sum() / (p2(n) * n).sum():.2f}; "
              f"12-bit: max bin mean {a[:, 5].mean():.1f} p90 {np.percentile(a[:, 5], 90):.0f}, sum sq / n {a[:, 6].sum() / n.sum():.1f}")


if __name__ == "__main__":
    main()


def tie_stats(kind="text", bs=1 << 20):
    """Round-1 ties of the wave / workgroup jobs for a key of K rotation bits after the job depth."""
    kid = {"text": bra.SYNTH_TEXT, "random": bra.SYNTH_RANDOM, "sym16": bra.SYNTH_SYM16}[kind]
    blk = bra.synth_fill(kid, bs, bs)
    keys, b = packed_bytes(blk)
    order = np.lexsort(keys.T[::-1])
    jobs, k = jobs_of(keys, order)
    for bits in (24, 32, 48, 56):
        nb = bits // 8
        tied = tot = 0
        gsz = []
        for s, e, d in jobs:
            if d + nb > NB:
                continue
            sub = k[s:e, d:d + nb]
            # rows equal to a neighbour (sorted order): tied after a round-1 key of `bits` bits
            eq = np.all(sub[1:] == sub[:-1], axis=1)
            t = np.zeros(e - s, bool)
            t[1:] |= eq
            t[:-1] |= eq
            tied += int(t.sum())
            tot += e - s
            # group sizes
            heads = np.concatenate([[True], ~eq])
            ids = np.cumsum(heads)
            cnt = np.bincount(ids)[1:]
            gsz.extend(cnt[cnt > 1].tolist())
        g = np.array(gsz) if gsz else np.array([0])
        print(f"{kind}: round-1 key of {bits} bits: tied {tied / max(1, tot):.1%} of {tot} job elements; tied groups {len(gsz)}, "
              f"mean size {g.mean():.1f}, p90 {np.percentile(g, 90):.0f}, max {g.max()}, elements in groups > 64: {g[g > 64].sum() / max(1, tot):.1%}")
