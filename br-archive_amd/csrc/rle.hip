// rle.hip -- PackBits run-length encoding for a batch of independent blocks.
//
// Replaces bra_rle_encode (reference src/encoders/bra_rle.c:60-120, size pre-scan :20-56, run
// detection :9-18).  The greedy reference encoder is restated in its structural (parallel) form,
// pinned against the reference by oracle/ (orc_rle_encode) and tests/golden:
//   * a maximal run of L >= 3 equal bytes becomes floor(L/128) run blocks of 128 and one run block
//     of r = L % 128 when r >= 3; for r in {1, 2} the r tail bytes are literals;
//   * literal positions form gaps; a gap is cut into literal blocks of <= 128 bytes from its start.
// Output bytes per input position: run-block start 2, run continuation 0, literal 1 (+1 control
// byte at gap offsets multiple of 128).  Positions are classified per 4 KiB tile with block-wide
// scans; cross-tile state (run extents, gap offsets, output offsets) comes from two tiny per-block
// sequential passes over tile summaries.
//   k_rle_runs    tile run summary (first/last byte, leading/trailing run, all-equal)
//   k_rle_link    per block: run extension into each tile from the left and from the right
//   k_rle_sizes   tile gap summary + output bytes excluding the leading gap's control bytes
//   k_rle_offsets per block: gap offset entering each tile, output offset, gap remainder after tile
//   k_rle_write   classify again, stage the tile's output in LDS, coalesced store, + byte histogram
//                 of the output (the Huffman frequencies, bra_huffman.c:368-370)
#include "rle.h"
#include "prof.h"

namespace bra {

namespace {

constexpr int TPB = 256;
constexpr int PT  = RLE_TILE / TPB;  // 16 bytes per thread

struct RunSum
{
    uint32_t len, pre, suf;
    uint8_t  first, last, all, pad;
};

__device__ __forceinline__ RunSum run_combine(const RunSum& A, const RunSum& B)
{
    if (A.len == 0)
        return B;
    if (B.len == 0)
        return A;
    RunSum R;
    R.len   = A.len + B.len;
    R.first = A.first;
    R.pre   = (A.all && A.first == B.first) ? A.len + B.pre : A.pre;
    R.last  = B.last;
    R.suf   = (B.all && B.last == A.last) ? B.len + A.suf : B.suf;
    R.all   = A.all && B.all && A.last == B.first;
    R.pad   = 0;
    return R;
}

struct GapSum
{
    uint32_t len, lead, trail, has;  // has = contains a non-literal position
};

__device__ __forceinline__ GapSum gap_combine(const GapSum& A, const GapSum& B)
{
    GapSum R;
    R.len   = A.len + B.len;
    R.has   = A.has | B.has;
    R.lead  = A.has ? A.lead : A.len + B.lead;
    R.trail = B.has ? B.trail : B.len + A.trail;
    return R;
}

__device__ __forceinline__ RunSum shfl_run(const RunSum& x, int src)
{
    RunSum r;
    r.len             = __shfl(x.len, src, 64);
    r.pre             = __shfl(x.pre, src, 64);
    r.suf             = __shfl(x.suf, src, 64);
    const uint32_t pk = __shfl((uint32_t) x.first | ((uint32_t) x.last << 8) | ((uint32_t) x.all << 16), src, 64);
    r.first           = pk & 0xFF;
    r.last            = (pk >> 8) & 0xFF;
    r.all             = (pk >> 16) & 1;
    r.pad             = 0;
    return r;
}

__device__ __forceinline__ GapSum shfl_gap(const GapSum& x, int src)
{
    return GapSum{(uint32_t) __shfl(x.len, src, 64), (uint32_t) __shfl(x.lead, src, 64), (uint32_t) __shfl(x.trail, src, 64),
                  (uint32_t) __shfl(x.has, src, 64)};
}

// Block-wide EXCLUSIVE scans over 256 threads (forward: combine(prefix, x); backward: combine(x, suffix)).
template <typename T, typename Comb, typename Shfl>
__device__ __forceinline__ T block_scan_fwd(const T& v, const T& seed, const T& ident, T* lds, Comb comb, Shfl shfl)
{
    const int lane = lane_id(), w = threadIdx.x >> 6;
    T         x    = v;
    for (int d = 1; d < 64; d <<= 1)
    {
        T o = shfl(x, max(lane - d, 0));
        if (lane >= d)
            x = comb(o, x);
    }
    if (lane == 63)
        lds[w] = x;
    T ex = shfl(x, max(lane - 1, 0));
    __syncthreads();
    T pre = seed;
    for (int i = 0; i < w; ++i)
        pre = comb(pre, lds[i]);
    __syncthreads();
    return lane == 0 ? pre : comb(pre, ex);
    (void) ident;
}

template <typename T, typename Comb, typename Shfl>
__device__ __forceinline__ T block_scan_bwd(const T& v, const T& seed, T* lds, Comb comb, Shfl shfl)
{
    const int lane = lane_id(), w = threadIdx.x >> 6;
    T         x    = v;
    for (int d = 1; d < 64; d <<= 1)
    {
        T o = shfl(x, min(lane + d, 63));
        if (lane + d < 64)
            x = comb(x, o);
    }
    if (lane == 0)
        lds[w] = x;
    T ex = shfl(x, min(lane + 1, 63));
    __syncthreads();
    T suf = seed;
    for (int i = 3; i > w; --i)
        suf = comb(lds[i], suf);
    __syncthreads();
    return lane == 63 ? suf : comb(ex, suf);
}

struct TileRun
{
    uint32_t len, pre, suf, flags;  // flags: first | last << 8 | all << 16
};

struct TileLink
{
    uint32_t left, right;  // run extension into the tile from before / after it
};

struct TileGap
{
    uint32_t lead, trail, has, fixed;
};

struct TileOff
{
    uint32_t g_in, out_off, rem_after, pad;
};

__device__ __forceinline__ void load16(const uint8_t* p, uint32_t cnt, uint32_t base, uint8_t (&x)[PT])
{
    // base = first tile byte of this thread; bytes beyond cnt are never used
    if (base + PT <= cnt && (((uintptr_t) (p + base)) & 15) == 0)
    {
        const uint4 v = *reinterpret_cast<const uint4*>(p + base);
        const uint32_t wds[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < PT; ++i)
            x[i] = (wds[i >> 2] >> (8 * (i & 3))) & 0xFF;
    }
    else
    {
#pragma unroll
        for (int i = 0; i < PT; ++i)
            x[i] = (base + i < cnt) ? p[base + i] : 0;
    }
}

// All per-thread loops below are fully unrolled over the PT positions (static register indices);
// positions >= n (tile end) are masked.
__device__ __forceinline__ uint32_t sel(const uint8_t (&x)[PT], uint32_t i)
{
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < PT; ++j)
        r = ((uint32_t) j == i) ? x[j] : r;
    return r;
}

__device__ __forceinline__ RunSum thread_runsum(const uint8_t (&x)[PT], uint32_t n)
{
    RunSum s;
    s.len = n;
    s.pad = 0;
    if (n == 0)
    {
        s.pre = s.suf = 0;
        s.first = s.last = 0;
        s.all            = 1;
        return s;
    }
    const uint32_t last = sel(x, n - 1);
    uint32_t       p = 1, q = 1;
    bool           pr = true, qr = true;
#pragma unroll
    for (int i = 1; i < PT; ++i)
    {
        pr = pr && (uint32_t) i < n && x[i] == x[0];
        p += pr ? 1 : 0;
    }
    // backwards from n-1: position n-1-j for j = 1..
#pragma unroll
    for (int i = PT - 2; i >= 0; --i)
    {
        const bool in = (uint32_t) i < n - 1;  // strictly before the last position
        // walk i = n-2, n-3, ... : positions above n-2 are skipped (not yet in the run walk)
        if (in)
        {
            qr = qr && x[i] == last;
            q += qr ? 1 : 0;
        }
    }
    s.first = x[0];
    s.last  = (uint8_t) last;
    s.pre   = p;
    s.suf   = q;
    s.all   = (p == n);
    return s;
}

// Per-position classification.  kind: 0 literal, 1 run-block start, 2 run continuation.
// For run-block starts clen = block length.  `left` / `right`: run extension into this thread's
// positions from before / after them (same byte as x[0] / x[n-1]).
__device__ __forceinline__ void classify(const uint8_t (&x)[PT], uint32_t n, uint32_t left, uint32_t right, uint8_t (&kind)[PT],
                                         uint8_t (&clen)[PT])
{
    uint32_t k[PT];  // position inside its maximal run
#pragma unroll
    for (int i = 0; i < PT; ++i)
        k[i] = (i == 0) ? left : (x[i] == x[i - 1] ? k[i - 1] + 1 : 0);
    uint32_t nxt = 0;
#pragma unroll
    for (int i = PT - 1; i >= 0; --i)
    {
        uint32_t r;  // positions from i to the end of its run, inclusive
        if ((uint32_t) i >= n)
            r = 0;
        else if ((uint32_t) i == n - 1)
            r = 1 + right;
        else
            r = (x[i] == x[i + 1]) ? nxt + 1 : 1;
        nxt                 = r;
        const uint32_t L    = k[i] + r;
        const uint32_t full = L >> 7, rm = L & 127, q = k[i] >> 7;
        uint8_t        kd = 0, cl = 0;
        if (L >= 3)
        {
            if (q < full)
            {
                kd = (k[i] & 127) == 0 ? 1 : 2;
                cl = 128;
            }
            else if (rm >= 3)
            {
                kd = (k[i] == (full << 7)) ? 1 : 2;
                cl = (uint8_t) rm;
            }
        }
        kind[i] = kd;
        clen[i] = cl;
    }
}

__device__ __forceinline__ GapSum thread_gapsum(const uint8_t (&kind)[PT], uint32_t n)
{
    GapSum   g{n, 0, 0, 0};
    bool     lead = true;
    uint32_t trail = 0;
#pragma unroll
    for (int i = 0; i < PT; ++i)
    {
        if ((uint32_t) i < n)
        {
            const bool lit = kind[i] == 0;
            lead           = lead && lit;
            g.lead += lead ? 1 : 0;
            g.has |= lit ? 0u : 1u;
            trail = lit ? trail + 1 : 0;
        }
    }
    g.trail = trail;
    return g;
}

__global__ void __launch_bounds__(TPB) k_rle_runs(const uint8_t* __restrict__ in, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                  TileRun* __restrict__ out)
{
    __shared__ RunSum lds[4];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const Piece    P = tiles[t];
        uint8_t        x[PT];
        const uint32_t base = threadIdx.x * PT;
        load16(in + P.off, P.len, base, x);
        const uint32_t n = base < P.len ? min((uint32_t) PT, P.len - base) : 0;
        RunSum         s = thread_runsum(x, n);
        RunSum         z{0, 0, 0, 0, 0, 0, 0};
        auto           comb = [](const RunSum& a, const RunSum& b) { return run_combine(a, b); };
        // inclusive total via exclusive + own
        RunSum ex  = block_scan_fwd(s, z, z, lds, comb, shfl_run);
        RunSum inc = run_combine(ex, s);
        if (threadIdx.x == TPB - 1)
            out[t] = TileRun{inc.len, inc.pre, inc.suf, (uint32_t) inc.first | ((uint32_t) inc.last << 8) | ((uint32_t) inc.all << 16)};
        __syncthreads();
    }
}

// One thread per block walks its tiles forward and backward.
__global__ void k_rle_link(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count, uint32_t nblocks,
                           const TileRun* __restrict__ tr, TileLink* __restrict__ link)
{
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += gridDim.x * blockDim.x)
    {
        const uint32_t t0 = first[b], nt = count[b];
        uint32_t       last = 0, suf = 0;
        for (uint32_t i = 0; i < nt; ++i)
        {
            const TileRun  T   = tr[t0 + i];
            const uint32_t fb  = T.flags & 0xFF, lb = (T.flags >> 8) & 0xFF, all = (T.flags >> 16) & 1;
            link[t0 + i].left  = (i > 0 && last == fb) ? suf : 0;
            suf                = (i > 0 && all && fb == last) ? suf + T.len : T.suf;
            last               = lb;
        }
        uint32_t firstb = 0, pre = 0;
        for (int i = (int) nt - 1; i >= 0; --i)
        {
            const TileRun  T   = tr[t0 + i];
            const uint32_t fb  = T.flags & 0xFF, lb = (T.flags >> 8) & 0xFF, all = (T.flags >> 16) & 1;
            link[t0 + i].right = (i < (int) nt - 1 && firstb == lb) ? pre : 0;
            pre                = (i < (int) nt - 1 && all && lb == firstb) ? pre + T.len : T.pre;
            firstb             = fb;
        }
    }
}

// Shared per-tile analysis: run classification, gap scans, output byte counts.
struct TileView
{
    uint8_t  x[PT];
    uint8_t  kind[PT];
    uint8_t  clen[PT];
    uint32_t n;
};

__device__ __forceinline__ void tile_classify(const uint8_t* __restrict__ in, const Piece& P, TileLink L, RunSum* lds, TileView& v)
{
    const uint32_t base = threadIdx.x * PT;
    load16(in + P.off, P.len, base, v.x);
    v.n      = base < P.len ? min((uint32_t) PT, P.len - base) : 0;
    RunSum s = thread_runsum(v.x, v.n);
    // seeds: the run entering from the left has the tile's first byte; from the right, its last byte
    __shared__ uint8_t edge[2];
    if (threadIdx.x == 0)
        edge[0] = v.x[0];
    if (base < P.len && base + v.n == P.len)
        edge[1] = (uint8_t) sel(v.x, v.n - 1);
    __syncthreads();
    RunSum sl{L.left, L.left, L.left, edge[0], edge[0], 1, 0};
    RunSum sr{L.right, L.right, L.right, edge[1], edge[1], 1, 0};
    auto   comb = [](const RunSum& a, const RunSum& b) { return run_combine(a, b); };
    RunSum E    = block_scan_fwd(s, sl, sl, lds, comb, shfl_run);
    RunSum F    = block_scan_bwd(s, sr, lds, comb, shfl_run);
    uint32_t left  = (v.n && E.len && E.last == v.x[0]) ? E.suf : 0;
    uint32_t right = (v.n && F.len && F.first == sel(v.x, v.n - 1)) ? F.pre : 0;
    classify(v.x, v.n, left, right, v.kind, v.clen);
}

// Output bytes of this thread's positions given the gap offset of its first position (go0) and
// the literal count following its last position (rem_after).  Optionally writes them to `stage`.
template <bool WRITE>
__device__ __forceinline__ uint32_t emit_thread(const TileView& v, uint32_t go0, uint32_t rem_after, uint8_t* stage, uint32_t pos)
{
    // remaining literals from position i to the gap end (inclusive), computed backwards
    uint32_t rem[PT];
    uint32_t run = rem_after;
#pragma unroll
    for (int i = PT - 1; i >= 0; --i)
    {
        if ((uint32_t) i < v.n)
            run = (v.kind[i] == 0) ? run + 1 : 0;
        rem[i] = run;
    }
    uint32_t go = go0, bytes = 0;
#pragma unroll
    for (int i = 0; i < PT; ++i)
    {
        if ((uint32_t) i >= v.n)
            continue;
        if (v.kind[i] == 0)
        {
            const bool ctl = (go & 127) == 0;
            if (WRITE)
            {
                if (ctl)
                    stage[pos + bytes] = (uint8_t) (min(rem[i], 128u) - 1);
                stage[pos + bytes + (ctl ? 1 : 0)] = v.x[i];
            }
            bytes += ctl ? 2 : 1;
            ++go;
        }
        else
        {
            go = 0;
            if (v.kind[i] == 1)
            {
                if (WRITE)
                {
                    stage[pos + bytes]     = (uint8_t) (int8_t) (1 - (int) v.clen[i]);
                    stage[pos + bytes + 1] = v.x[i];
                }
                bytes += 2;
            }
        }
    }
    return bytes;
}

__global__ void __launch_bounds__(TPB) k_rle_sizes(const uint8_t* __restrict__ in, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                   const TileLink* __restrict__ link, TileGap* __restrict__ tg)
{
    __shared__ RunSum   lds[4];
    __shared__ GapSum   glds[4];
    __shared__ uint32_t tmp[8];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const Piece P = tiles[t];
        TileView    v;
        tile_classify(in, P, link[t], lds, v);
        const GapSum gs   = thread_gapsum(v.kind, v.n);
        auto         comb = [](const GapSum& a, const GapSum& b) { return gap_combine(a, b); };
        const GapSum z{0, 0, 0, 0};
        const GapSum E = block_scan_fwd(gs, z, z, glds, comb, shfl_gap);
        const GapSum F = block_scan_bwd(gs, z, glds, comb, shfl_gap);
        const uint32_t bytes = emit_thread<false>(v, E.trail, F.lead, nullptr, 0);
        uint32_t       total;
        block256_exclusive_sum(bytes, tmp, &total);
        if (threadIdx.x == TPB - 1)
        {
            const GapSum tot = gap_combine(E, gs);
            // leading stretch control bytes were counted with gap offset 0: ceil(lead/128)
            tg[t] = TileGap{tot.lead, tot.trail, tot.has, total - (tot.lead + 127) / 128};
        }
        __syncthreads();
    }
}

__global__ void k_rle_offsets(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count, uint32_t nblocks,
                              const Piece* __restrict__ tiles, const TileGap* __restrict__ tg, TileOff* __restrict__ to,
                              uint32_t* __restrict__ rle_size)
{
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += gridDim.x * blockDim.x)
    {
        const uint32_t t0 = first[b], nt = count[b];
        uint32_t       g = 0, run = 0;
        for (uint32_t i = 0; i < nt; ++i)
        {
            const TileGap  G    = tg[t0 + i];
            const uint32_t ctrl = (g + G.lead + 127) / 128 - (g + 127) / 128;
            to[t0 + i].g_in     = g;
            to[t0 + i].out_off  = run;
            run += G.fixed + ctrl;
            g = G.has ? G.trail : g + G.lead;
        }
        rle_size[b]  = run;
        uint32_t rem = 0;
        for (int i = (int) nt - 1; i >= 0; --i)
        {
            to[t0 + i].rem_after = rem;
            const TileGap G      = tg[t0 + i];
            rem                  = G.has ? G.lead : tiles[t0 + i].len + rem;
        }
    }
}

__global__ void __launch_bounds__(TPB) k_rle_write(const uint8_t* __restrict__ in, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                   const TileLink* __restrict__ link, const TileOff* __restrict__ to,
                                                   const uint64_t* __restrict__ rle_base, uint8_t* __restrict__ out,
                                                   uint32_t* __restrict__ hist)
{
    __shared__ RunSum   lds[4];
    __shared__ GapSum   glds[4];
    __shared__ uint32_t tmp[8];
    __shared__ uint8_t  stage[RLE_TILE + RLE_TILE / 64 + 64];
    __shared__ uint32_t h[256];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const Piece   P = tiles[t];
        const TileOff O = to[t];
        h[threadIdx.x]  = 0;
        TileView v;
        tile_classify(in, P, link[t], lds, v);
        const GapSum gs   = thread_gapsum(v.kind, v.n);
        auto         comb = [](const GapSum& a, const GapSum& b) { return gap_combine(a, b); };
        const GapSum z{0, 0, 0, 0};
        const GapSum sl{O.g_in, O.g_in, O.g_in, 0};
        const GapSum sr{O.rem_after, O.rem_after, O.rem_after, 0};
        const GapSum E     = block_scan_fwd(gs, sl, z, glds, comb, shfl_gap);
        const GapSum F     = block_scan_bwd(gs, sr, glds, comb, shfl_gap);
        const uint32_t by  = emit_thread<false>(v, E.trail, F.lead, nullptr, 0);
        uint32_t       total;
        const uint32_t pos = block256_exclusive_sum(by, tmp, &total);
        emit_thread<true>(v, E.trail, F.lead, stage, pos);
        __syncthreads();
        uint8_t* dst = out + rle_base[P.block] + O.out_off;
        for (uint32_t i = threadIdx.x; i < total; i += TPB)
        {
            const uint8_t c = stage[i];
            dst[i]          = c;
            atomicAdd(&h[c], 1u);
        }
        __syncthreads();
        if (h[threadIdx.x])
            atomicAdd(&hist[(size_t) P.block * 256 + threadIdx.x], h[threadIdx.x]);
        __syncthreads();
    }
}

}  // namespace

bool rle_encode_device(RleWorkspace& w, const uint8_t* d_in, const BlockDesc* h_blocks, uint32_t nblocks, const uint64_t* d_rle_base,
                       uint8_t* d_out, uint32_t* d_rle_size, uint32_t* d_hist, hipStream_t s)
{
    if (!w.tiling.build(h_blocks, nblocks, RLE_TILE, s))
        return false;
    const uint32_t nt = w.tiling.n;
    if (!w.reserve(nt))
        return false;
    const uint32_t grid = std::min<uint32_t>(nt, 8192);
    BRA_HIP_CHECK(hipMemsetAsync(d_hist, 0, (size_t) nblocks * 256 * 4, s));
    TileRun*  runs = static_cast<TileRun*>(w.runs);
    TileLink* link = static_cast<TileLink*>(w.link);
    TileGap*  gaps = static_cast<TileGap*>(w.gaps);
    TileOff*  offs = static_cast<TileOff*>(w.offs);
    {
        BRA_PROF(P_RLE_RUNS, s);
        hipLaunchKernelGGL(k_rle_runs, dim3(grid), dim3(TPB), 0, s, d_in, w.tiling.d_pieces, nt, runs);
    }
    {
        BRA_PROF(P_RLE_LINK, s);
        hipLaunchKernelGGL(k_rle_link, dim3(div_up(nblocks, 64)), dim3(64), 0, s, w.tiling.d_first, w.tiling.d_count, nblocks, runs, link);
    }
    {
        BRA_PROF(P_RLE_SIZES, s);
        hipLaunchKernelGGL(k_rle_sizes, dim3(grid), dim3(TPB), 0, s, d_in, w.tiling.d_pieces, nt, link, gaps);
    }
    {
        BRA_PROF(P_RLE_OFFSETS, s);
        hipLaunchKernelGGL(k_rle_offsets, dim3(div_up(nblocks, 64)), dim3(64), 0, s, w.tiling.d_first, w.tiling.d_count, nblocks,
                           w.tiling.d_pieces, gaps, offs, d_rle_size);
    }
    {
        BRA_PROF(P_RLE_WRITE, s);
        hipLaunchKernelGGL(k_rle_write, dim3(grid), dim3(TPB), 0, s, d_in, w.tiling.d_pieces, nt, link, offs, d_rle_base, d_out, d_hist);
    }
    if (g_prof && g_prof->mask)
    {
        // rle.write (n + r bytes) is charged by the caller once the output sizes are on the host
        uint64_t N = 0;
        for (uint32_t b = 0; b < nblocks; ++b)
            N += h_blocks[b].len;
        prof_bytes(P_RLE_RUNS, (double) N + 16.0 * nt);
        prof_bytes(P_RLE_SIZES, (double) N + 24.0 * nt);
        prof_bytes(P_RLE_LINK, 24.0 * nt);
        prof_bytes(P_RLE_OFFSETS, 48.0 * nt);
    }
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

bool RleWorkspace::reserve(uint32_t ntiles)
{
    if (ntiles <= cap)
        return true;
    (void) hipFree(runs);
    (void) hipFree(link);
    (void) hipFree(gaps);
    (void) hipFree(offs);
    cap = ntiles + ntiles / 4 + 64;
    BRA_HIP_CHECK(hipMalloc(&runs, cap * 16));
    BRA_HIP_CHECK(hipMalloc(&link, cap * 8));
    BRA_HIP_CHECK(hipMalloc(&gaps, cap * 16));
    BRA_HIP_CHECK(hipMalloc(&offs, cap * 16));
    return true;
}

void RleWorkspace::release()
{
    tiling.release();
    (void) hipFree(runs);
    (void) hipFree(link);
    (void) hipFree(gaps);
    (void) hipFree(offs);
    runs = link = gaps = offs = nullptr;
    cap                       = 0;
}

}  // namespace bra
