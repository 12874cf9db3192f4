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
#include "rle_tile.h"

namespace bra {

namespace {

using namespace rle_tile;  // per-thread classification and output (PT positions per thread)
constexpr int TPB = 256;
static_assert(RLE_TILE == TPB * PT, "one tile per workgroup, PT positions per thread");

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

// Exclusive scan over the 256 threads of the workgroup (thread order FWD or reversed), seeded
// with `seed` (the value before the first / after the last thread).  tmp: 4 dwords of LDS.  If
// `total` is given it receives the inclusive total including the seed.
template <bool FWD, typename Op>
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t seed, uint32_t id, Op op, uint32_t* tmp, uint32_t* total = nullptr)
{
    const int      lane = lane_id(), w = (int) wave_id();
    uint32_t       ex;  // scan of the lanes before this one in scan order (id at the wave's first lane)
    const uint32_t inc = wave_scan<FWD>(v, id, op, &ex);
    if (lane == (FWD ? 63 : 0))
        tmp[w] = inc;
    __syncthreads();
    uint32_t pre = seed, all = seed;
#pragma unroll
    for (int i = 0; i < 4; ++i)
    {
        const int      k = FWD ? i : 3 - i;
        const uint32_t t = tmp[k];
        if (FWD ? (k < w) : (k > w))
            pre = op(pre, t);
        all = op(all, t);
    }
    __syncthreads();
    if (total)
        *total = all;
    return op(pre, ex);
}

// Two independent exclusive workgroup scans (orders F1 / F2, seeds, identities as block_scan_excl)
// sharing one LDS exchange and ONE barrier: tmp = 8 dwords that no thread touches again before the
// caller's next barrier (callers rotate three regions, so a tile costs one barrier per dependent
// scan round instead of two per scan).  all1 / all2 receive the totals including the seeds.
template <bool F1, bool F2, typename O1, typename O2>
__device__ __forceinline__ void block_scan_pair(uint32_t v1, uint32_t seed1, uint32_t id1, O1 op1, uint32_t& ex1, uint32_t& all1, uint32_t v2,
                                                uint32_t seed2, uint32_t id2, O2 op2, uint32_t& ex2, uint32_t& all2, uint32_t* tmp)
{
    const int      lane = lane_id(), w = (int) wave_id();
    uint32_t       e1, e2;
    const uint32_t i1 = wave_scan<F1>(v1, id1, op1, &e1);
    const uint32_t i2 = wave_scan<F2>(v2, id2, op2, &e2);
    if (lane == (F1 ? 63 : 0))
        tmp[w] = i1;
    if (lane == (F2 ? 63 : 0))
        tmp[4 + w] = i2;
    __syncthreads();
    uint32_t p1 = seed1, a1 = seed1, p2 = seed2, a2 = seed2;
#pragma unroll
    for (int i = 0; i < 4; ++i)
    {
        const int      k1 = F1 ? i : 3 - i, k2 = F2 ? i : 3 - i;
        const uint32_t t1 = tmp[k1], t2 = tmp[4 + k2];
        if (F1 ? (k1 < w) : (k1 > w))
            p1 = op1(p1, t1);
        if (F2 ? (k2 < w) : (k2 > w))
            p2 = op2(p2, t2);
        a1 = op1(a1, t1);
        a2 = op2(a2, t2);
    }
    ex1  = op1(p1, e1);
    ex2  = op2(p2, e2);
    all1 = a1;
    all2 = a2;
}

// Exclusive sum over the workgroup with one barrier (tmp as in block_scan_pair: 4 dwords).
__device__ __forceinline__ uint32_t block_sum_excl1(uint32_t v, uint32_t* tmp, uint32_t& total)
{
    const int      lane = lane_id(), w = (int) wave_id();
    const uint32_t x    = wave_scan<true>(v, 0u, OpAdd());
    if (lane == 63)
        tmp[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
    {
        const uint32_t t = tmp[i];
        if (i < w)
            pre += t;
        tot += t;
    }
    total = tot;
    return pre + x - v;
}

// One tile as the workgroup sees it: thread t holds positions [16t, 16t + nt) of the tile.
struct TileThread
{
    uint32_t w[4];
    uint32_t base, nt, n;
    uint32_t bm;    // run boundaries at the thread's positions (position 0 of the tile always is one)
};

__device__ __forceinline__ void tile_load(const uint8_t* __restrict__ in, const Piece& P, TileThread& T)
{
    const uint8_t* p = in + P.off;
    T.n              = P.len;
    T.base           = threadIdx.x * PT;
    T.nt             = T.base < T.n ? min((uint32_t) PT, T.n - T.base) : 0;
    if (T.nt == PT && (((uintptr_t) (p + T.base)) & 15) == 0)
    {
        const uint4 v = *reinterpret_cast<const uint4*>(p + T.base);
        T.w[0] = v.x, T.w[1] = v.y, T.w[2] = v.z, T.w[3] = v.w;
    }
    else
    {
#pragma unroll
        for (int d = 0; d < 4; ++d)
        {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (T.base + 4 * d + j < T.n)
                    x |= (uint32_t) p[T.base + 4 * d + j] << (8 * j);
            T.w[d] = x;
        }
    }
    const uint32_t prev = T.base > 0 && T.nt ? p[T.base - 1] : 0u;
    uint32_t       bm   = diff_mask(T.w, prev);
    if (T.base == 0)
        bm |= 1u;
    T.bm = T.nt ? bm & ((1u << T.nt) - 1u) : 0u;
}

// Run classification of the thread's positions (rle_tile.h) from the boundary scans.
__device__ __forceinline__ RunCls tile_cls(const TileThread& T, uint32_t left, uint32_t right, uint32_t* tmp)
{
    uint32_t Sprev, Enext, u0, u1;
    block_scan_pair<true, false>(T.bm ? T.base + hi_bit(T.bm) : 0u, 0u, 0u, OpMax(), Sprev, u0, T.bm ? T.base + lo_bit(T.bm) : T.n, T.n, T.n,
                                 OpMin(), Enext, u1, tmp);
    return cls_thread(T.bm, T.nt, T.base, T.n, Sprev, Enext, left, right);
}

// Tile run summary: leading / trailing run length, first / last byte, all one run.
__global__ void __launch_bounds__(TPB) k_rle_runs(const uint8_t* __restrict__ in, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                  TileRun* __restrict__ out)
{
    __shared__ uint32_t tmp[8];
    __shared__ uint32_t edge[2];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const Piece P = tiles[t];
        TileThread  T;
        tile_load(in, P, T);
        if (T.nt && T.base + T.nt == T.n)
            edge[1] = byte_at(T.w, (int) T.nt - 1);
        if (threadIdx.x == 0)
            edge[0] = byte_at(T.w, 0);
        // first boundary after position 0 and the last boundary (one scan pair: edge[] is read
        // after its barrier)
        const uint32_t b1 = T.bm & ~(T.base == 0 ? 1u : 0u);
        uint32_t       lo, hi, u0, u1;
        block_scan_pair<true, true>(T.bm ? T.base + hi_bit(T.bm) : 0u, 0u, 0u, OpMax(), u0, hi, b1 ? T.base + lo_bit(b1) : T.n, T.n, T.n, OpMin(),
                                    u1, lo, tmp);
        if (threadIdx.x == 0)
        {
            const uint32_t all = lo >= T.n ? 1u : 0u;
            out[t]             = TileRun{T.n, lo, T.n - hi, edge[0] | (edge[1] << 8) | (all << 16)};
        }
        __syncthreads();
    }
}

// Run summary of a stretch of tiles (the run monoid): length, first / last byte, leading /
// trailing run length, all one run.
struct RunSum
{
    uint32_t len, pre, suf, first, last, all;
};

__device__ __forceinline__ RunSum run_combine(const RunSum& A, const RunSum& B)
{
    if (A.len == 0)
        return B;
    if (B.len == 0)
        return A;
    const bool join = A.last == B.first;
    return RunSum{A.len + B.len, (A.all && join) ? A.len + B.pre : A.pre, (B.all && join) ? B.len + A.suf : B.suf, A.first, B.last,
                  (A.all && B.all && join) ? 1u : 0u};
}

__device__ __forceinline__ RunSum shfl_run(const RunSum& x, int src)
{
    return RunSum{(uint32_t) __shfl((int) x.len, src, 64), (uint32_t) __shfl((int) x.pre, src, 64), (uint32_t) __shfl((int) x.suf, src, 64),
                  (uint32_t) __shfl((int) x.first, src, 64), (uint32_t) __shfl((int) x.last, src, 64), (uint32_t) __shfl((int) x.all, src, 64)};
}

// Gap-offset recurrence g -> h ? v : g + v of one tile (or a stretch of tiles: composition).
struct GapFn
{
    uint32_t h, v;
};

__device__ __forceinline__ GapFn gap_then(const GapFn& a, const GapFn& b) { return b.h ? b : GapFn{a.h, a.v + b.v}; }

__device__ __forceinline__ GapFn shfl_gap(const GapFn& x, int src)
{
    return GapFn{(uint32_t) __shfl((int) x.h, src, 64), (uint32_t) __shfl((int) x.v, src, 64)};
}

// Inclusive scan across the 64 lanes of a wave with a generic combine (lane order FWD or reversed):
// comb(earlier, later) in scan order.
template <bool FWD, typename T, typename Comb, typename Shfl>
__device__ __forceinline__ T wave_scan_t(T x, Comb comb, Shfl shfl)
{
    const int lane = lane_id();
    for (int d = 1; d < 64; d <<= 1)
    {
        const T o = shfl(x, FWD ? max(lane - d, 0) : min(lane + d, 63));
        if (FWD ? lane >= d : lane + d < 64)
            x = FWD ? comb(o, x) : comb(x, o);
    }
    return x;
}

// One wave per block: run extension into every tile from the left and from the right.
__global__ void __launch_bounds__(64) k_rle_link(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count, uint32_t nblocks,
                                                 const TileRun* __restrict__ tr, TileLink* __restrict__ link)
{
    const int  lane  = lane_id();
    const auto comb  = [](const RunSum& a, const RunSum& b) { return run_combine(a, b); };
    const auto load  = [&](uint32_t t) {
        const TileRun T = tr[t];
        return RunSum{T.len, T.pre, T.suf, T.flags & 0xFFu, (T.flags >> 8) & 0xFFu, (T.flags >> 16) & 1u};
    };
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t t0 = first[b], nt = count[b];
        RunSum         carry{0, 0, 0, 0, 0, 1};  // tiles before the chunk
        for (uint32_t c = 0; c < nt; c += 64)
        {
            const uint32_t i   = c + lane;
            const RunSum   me  = i < nt ? load(t0 + i) : RunSum{0, 0, 0, 0, 0, 1};
            const RunSum   inc = wave_scan_t<true>(me, comb, shfl_run);
            RunSum         ex  = shfl_run(inc, max(lane - 1, 0));
            ex                 = lane == 0 ? carry : run_combine(carry, ex);
            if (i < nt)
                link[t0 + i].left = (ex.len && ex.last == me.first) ? ex.suf : 0u;
            carry = run_combine(carry, shfl_run(inc, 63));
        }
        carry = RunSum{0, 0, 0, 0, 0, 1};  // tiles after the chunk
        for (int c = (int) ((nt + 63) / 64) * 64 - 64; c >= 0; c -= 64)
        {
            const uint32_t i   = (uint32_t) c + lane;
            const RunSum   me  = i < nt ? load(t0 + i) : RunSum{0, 0, 0, 0, 0, 1};
            const RunSum   inc = wave_scan_t<false>(me, comb, shfl_run);
            RunSum         ex  = shfl_run(inc, min(lane + 1, 63));
            ex                 = lane == 63 ? carry : run_combine(ex, carry);
            if (i < nt)
                link[t0 + i].right = (ex.len && ex.first == me.last) ? ex.pre : 0u;
            carry = run_combine(shfl_run(inc, 0), carry);
        }
    }
}

__global__ void __launch_bounds__(TPB) k_rle_sizes(const uint8_t* __restrict__ in, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                   const TileLink* __restrict__ link, TileGap* __restrict__ tg)
{
    __shared__ uint32_t tmp[3][8];  // one region per dependent scan round (block_scan_pair)
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const Piece    P = tiles[t];
        const TileLink K = link[t];
        TileThread     T;
        tile_load(in, P, T);
        const RunCls C = tile_cls(T, K.left, K.right, tmp[0]);
        const uint32_t nl = C.nl;
        uint32_t maxNL, minNL, GSprev, u0;
        block_scan_pair<true, true>(nl ? T.base + hi_bit(nl) + 1 : 0u, 0u, 0u, OpMax(), GSprev, maxNL, nl ? T.base + lo_bit(nl) : T.n, T.n, T.n,
                                    OpMin(), u0, minNL, tmp[1]);
        const uint32_t bytes = out_bytes(C, T.nt, T.base, GSprev, 0u);
        uint32_t       total;
        block_sum_excl1(bytes, tmp[2], total);
        if (threadIdx.x == 0)
        {
            const uint32_t has  = maxNL > 0 ? 1u : 0u;
            const uint32_t lead = has ? minNL : T.n;
            // the leading stretch's control bytes were counted with gap offset 0: ceil(lead/128)
            tg[t] = TileGap{lead, has ? T.n - maxNL : T.n, has, total - (lead + 127) / 128};
        }
    }
}

// One wave per block: gap offset entering each tile, output offset, literals after the tile.
__global__ void __launch_bounds__(64) k_rle_offsets(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count, uint32_t nblocks,
                                                    const Piece* __restrict__ tiles, const TileGap* __restrict__ tg, TileOff* __restrict__ to,
                                                    uint32_t* __restrict__ rle_size)
{
    const int  lane = lane_id();
    const auto fwd  = [](const GapFn& a, const GapFn& b) { return gap_then(a, b); };
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t t0 = first[b], nt = count[b];
        GapFn          carry{0, 0};
        uint32_t       run = 0;
        for (uint32_t c = 0; c < nt; c += 64)
        {
            const uint32_t i = c + lane;
            TileGap        G{0, 0, 0, 0};
            if (i < nt)
                G = tg[t0 + i];
            const GapFn    me  = i < nt ? GapFn{G.has, G.has ? G.trail : G.lead} : GapFn{0, 0};
            const GapFn    inc = wave_scan_t<true>(me, fwd, shfl_gap);
            GapFn          ex  = shfl_gap(inc, max(lane - 1, 0));
            ex                 = lane == 0 ? carry : gap_then(carry, ex);
            const uint32_t g    = ex.v;  // the recurrence starts from g = 0
            const uint32_t cost = i < nt ? G.fixed + (g + G.lead + 127) / 128 - (g + 127) / 128 : 0u;
            const uint32_t csum = wave_scan<true>(cost, 0u, OpAdd());
            if (i < nt)
            {
                to[t0 + i].g_in    = g;
                to[t0 + i].out_off = run + csum - cost;
            }
            run += __builtin_amdgcn_readlane(csum, 63);
            carry = gap_then(carry, shfl_gap(inc, 63));
        }
        if (lane == 0)
            rle_size[b] = run;
        // literals after each tile: rem -> has ? lead : len + rem, applied from the block end
        GapFn rc{0, 0};
        for (int c = (int) ((nt + 63) / 64) * 64 - 64; c >= 0; c -= 64)
        {
            const uint32_t i = (uint32_t) c + lane;
            GapFn          me{0, 0};
            if (i < nt)
            {
                const TileGap G = tg[t0 + i];
                me              = GapFn{G.has, G.has ? G.lead : tiles[t0 + i].len};
            }
            // composition in reverse: apply later tiles first
            const auto  bwd = [](const GapFn& a, const GapFn& b) { return gap_then(b, a); };
            const GapFn inc = wave_scan_t<false>(me, bwd, shfl_gap);
            GapFn       ex  = shfl_gap(inc, min(lane + 1, 63));
            ex              = lane == 63 ? rc : gap_then(rc, ex);
            if (i < nt)
                to[t0 + i].rem_after = ex.v;
            rc = gap_then(rc, shfl_gap(inc, 0));
        }
    }
}

__global__ void __launch_bounds__(TPB) k_rle_write(const uint8_t* __restrict__ in, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                   const TileLink* __restrict__ link, const TileOff* __restrict__ to,
                                                   const uint64_t* __restrict__ rle_base, uint8_t* __restrict__ out,
                                                   uint32_t* __restrict__ hist)
{
    __shared__ uint32_t tmp[2][8];  // tile_cls' scan pair, then the two-barrier scans
    __shared__ uint8_t  stage[RLE_TILE + RLE_TILE / 64 + 64];
    constexpr int       HC = 4, HS = 256 + 16;  // histogram copies (lane & 3), 16 banks apart: output bytes are skewed
    __shared__ uint32_t h[HC * HS];
    const XcdTiles X = xcd_tiles(ntiles);
    for (uint32_t t = X.t; t < X.end; t += X.step)
    {
        const Piece    P = tiles[t];
        const TileOff  O = to[t];
        const TileLink K = link[t];
#pragma unroll
        for (int c = 0; c < HC; ++c)
            h[c * HS + threadIdx.x] = 0;
        TileThread T;
        tile_load(in, P, T);
        const RunCls   C      = tile_cls(T, K.left, K.right, tmp[0]);
        const uint32_t nl     = C.nl;
        const uint32_t GSprev = block_scan_excl<true>(nl ? T.base + hi_bit(nl) + 1 : 0u, 0u, 0u, OpMax(), tmp[1]);
        const uint32_t GEnext = block_scan_excl<false>(nl ? T.base + lo_bit(nl) : T.n, T.n, T.n, OpMin(), tmp[1]);
        const uint32_t by     = out_bytes(C, T.nt, T.base, GSprev, O.g_in);
        uint32_t       total;
        const uint32_t pos = block256_exclusive_sum(by, tmp[1], &total);
        stage_out(T.w, T.bm, C, T.nt, T.base, T.n, GSprev, GEnext, O.g_in, O.rem_after, stage, pos);
        __syncthreads();
        uint8_t*       dst = out + rle_base[P.block] + O.out_off;
        const uint32_t cp  = (uint32_t) (lane_id() & (HC - 1)) * HS;
        for (uint32_t i = threadIdx.x; i < total; i += TPB)
        {
            const uint8_t c = stage[i];
            dst[i]          = c;
            atomicAdd(&h[cp + c], 1u);
        }
        __syncthreads();
        uint32_t hv = 0;
#pragma unroll
        for (int c = 0; c < HC; ++c)
            hv += h[c * HS + threadIdx.x];
        if (hv)
            atomicAdd(&hist[(size_t) P.block * 256 + threadIdx.x], hv);
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
    const uint32_t grid = std::min<uint32_t>(nt, 32768u);  // workgroups of the tile kernels (8192: 0.03 ms slower per stage)
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
        hipLaunchKernelGGL(k_rle_link, dim3(std::min<uint32_t>(nblocks, 4096)), dim3(64), 0, s, w.tiling.d_first, w.tiling.d_count, nblocks, runs, link);
    }
    {
        BRA_PROF(P_RLE_SIZES, s);
        hipLaunchKernelGGL(k_rle_sizes, dim3(grid), dim3(TPB), 0, s, d_in, w.tiling.d_pieces, nt, link, gaps);
    }
    {
        BRA_PROF(P_RLE_OFFSETS, s);
        hipLaunchKernelGGL(k_rle_offsets, dim3(std::min<uint32_t>(nblocks, 4096)), dim3(64), 0, s, w.tiling.d_first, w.tiling.d_count, nblocks,
                           w.tiling.d_pieces, gaps, offs, d_rle_size);
    }
    {
        BRA_PROF(P_RLE_WRITE, s);
        hipLaunchKernelGGL(k_rle_write, dim3(xcd_grid(grid)), dim3(TPB), 0, s, d_in, w.tiling.d_pieces, nt, link, offs, d_rle_base, d_out, d_hist);
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
    cap              = 0;
    const uint64_t c = ntiles + ntiles / 4 + 64;
    if (!dev_alloc_bytes(runs, c * 16) || !dev_alloc_bytes(link, c * 8) || !dev_alloc_bytes(gaps, c * 16) || !dev_alloc_bytes(offs, c * 16))
        return false;
    cap = (uint32_t) c;
    return true;
}

bool RleWorkspace::reserve_decode(uint64_t bytes)
{
    if (bytes <= dmap_cap)
        return true;
    dmap_cap         = 0;
    const uint64_t c = bytes + bytes / 4 + 4096;
    if (!dev_alloc_bytes(dmap, c))
        return false;
    dmap_cap = c;
    return true;
}

void RleWorkspace::release()
{
    tiling.release();
    (void) hipFree(dmap);
    dmap     = nullptr;
    dmap_cap = 0;
    (void) hipFree(runs);
    (void) hipFree(link);
    (void) hipFree(gaps);
    (void) hipFree(offs);
    runs = link = gaps = offs = nullptr;
    cap                       = 0;
}

}  // namespace bra
