// bwt_large.hip -- BWT of one block of 2^24 bytes or more (the single-block C-ABI bra_bwt_encode2,
// /root/reference/src/encoders/bra_bwt.c:73-108, takes any u32 length; the batched MSD/job path
// packs 24-bit rotation indices into its payloads and stops at 2^24).
//
// Prefix doubling over cyclic rotations: after the pass with offset h every rotation carries the
// rank of its first 2h bytes (the number of rotations whose first 2h bytes are smaller).  A pass
// builds key(i) = rank(i) << B | rank((i + h) mod n), B = ceil(log2 n) bits, for i in index order,
// sorts the (key, i) pairs with the stable LSD radix sort below (tied rotations stay in index
// order, the glibc qsort_r merge-sort tie rule of the reference), and assigns each rotation the
// start of its key's run (head flags + max-scan).  It stops once every key is distinct or 2h >= n
// (identical rotations of a periodic block).  L[j] = in[(sa[j] + n - 1) mod n], pi = the slot
// holding rotation 0.
//
// The sort is hand-written: 8-bit digits, one pass per digit of the 2B key bits, each pass
//   k_rs_hist     per 4096-element tile: digit counts in LDS -> hist[digit][tile] (digit-major),
//   scan          exclusive sum over hist (k_scan_reduce / k_scan_top / k_scan_apply),
//   k_rs_scatter  per tile, 16 rounds of 256 elements in index order: the stable rank of each
//                 element among the tile's equal digits (wave match by 8 ballots, per-wave counts
//                 through LDS, running digit counters across rounds) + its digit's tile offset.
// HBM traffic per pass ~ 2 x 12 B per element; text blocks of 16-64 MiB finish in 6-10 doubling
// passes.  This path is for correctness at large sizes, not the benchmark shape.
#include "bwt.h"

#include <algorithm>

namespace bra {
namespace {

constexpr uint32_t LG_TPB  = 256;
constexpr uint32_t LG_PT   = 16;
constexpr uint32_t LG_TILE = LG_TPB * LG_PT;  // elements per radix tile / scan block

// grid-strided loops over u32 element ranges with a 64-bit index (no wrap near 2^32)
#define LG_FOR(i, n) for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (uint64_t) gridDim.x * blockDim.x)

// pass 0: key(i) = in[i] << B | in[(i + 1) mod n] (the first two bytes of rotation i)
__global__ void k_lg_keys0(const uint8_t* __restrict__ in, uint32_t n, uint32_t B, uint64_t* __restrict__ key, uint32_t* __restrict__ idx)
{
    LG_FOR(i, n)
    {
        const uint64_t j = i + 1 == n ? 0 : i + 1;
        key[i]           = ((uint64_t) in[i] << B) | in[j];
        idx[i]           = (uint32_t) i;
    }
}

// pass h: key(i) = rank[i] << B | rank[(i + h) mod n]
__global__ void k_lg_keys(const uint32_t* __restrict__ rank, uint32_t n, uint32_t h, uint32_t B, uint64_t* __restrict__ key,
                          uint32_t* __restrict__ idx)
{
    LG_FOR(i, n)
    {
        const uint64_t j = i + h;
        key[i]           = ((uint64_t) rank[i] << B) | rank[j >= n ? j - n : j];
        idx[i]           = (uint32_t) i;
    }
}

// head[j] = j at the start of a run of equal keys, else 0; *tied = 1 if any run has length > 1
__global__ void k_lg_heads(const uint64_t* __restrict__ key, uint32_t n, uint32_t* __restrict__ head, uint32_t* __restrict__ tied)
{
    LG_FOR(j, n)
    {
        const bool h = j == 0 || key[j] != key[j - 1];
        head[j]      = h ? (uint32_t) j : 0u;
        if (!h)
            *tied = 1u;  // plain vector store; every writer stores the same value
    }
}

__global__ void k_lg_rank(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ grp, uint32_t n, uint32_t* __restrict__ rank)
{
    LG_FOR(j, n)
    rank[sa[j]] = grp[j];
}

__global__ void k_lg_emit(const uint8_t* __restrict__ in, const uint32_t* __restrict__ sa, uint32_t n, uint8_t* __restrict__ L,
                          uint32_t* __restrict__ pi)
{
    LG_FOR(j, n)
    {
        const uint32_t r = sa[j];
        L[j]             = in[r == 0 ? n - 1 : r - 1];
        if (r == 0)
            *pi = (uint32_t) j;
    }
}

// ---- device scans over u32 arrays (exclusive sum or inclusive max), three kernels ----
template <bool MAX>
__device__ __forceinline__ uint32_t scan_op(uint32_t a, uint32_t b) { return MAX ? max(a, b) : a + b; }

// Tile scan of LG_TILE values (16 consecutive per thread) with carry-in c, written back in place
// (when `write`) as an exclusive (EXCL) or inclusive scan; returns the tile's total (without c).
template <bool MAX, bool EXCL>
__device__ __forceinline__ uint32_t tile_scan(uint32_t* __restrict__ a, uint64_t base, uint64_t n, uint32_t c, bool write)
{
    __shared__ uint32_t part[LG_TPB / 64];
    uint32_t            v[LG_PT], s = 0;
    const uint64_t      i0 = base + (uint64_t) threadIdx.x * LG_PT;
#pragma unroll
    for (uint32_t k = 0; k < LG_PT; ++k)
    {
        v[k] = i0 + k < n ? a[i0 + k] : 0u;
        s    = scan_op<MAX>(s, v[k]);
    }
    uint32_t       ex;
    const uint32_t inc = MAX ? wave_scan<true>(s, 0u, OpMax(), &ex) : wave_scan<true>(s, 0u, OpAdd(), &ex);
    const uint32_t w   = threadIdx.x >> 6;
    if (lane_id() == 63)
        part[w] = inc;
    __syncthreads();
    uint32_t pre = c, tot = 0;
    for (uint32_t q = 0; q < LG_TPB / 64; ++q)
    {
        if (q < w)
            pre = scan_op<MAX>(pre, part[q]);
        tot = scan_op<MAX>(tot, part[q]);
    }
    __syncthreads();
    if (write)
    {
        uint32_t run = scan_op<MAX>(pre, ex);
#pragma unroll
        for (uint32_t k = 0; k < LG_PT; ++k)
        {
            const uint32_t nx = scan_op<MAX>(run, v[k]);
            if (i0 + k < n)
                a[i0 + k] = EXCL ? run : nx;
            run = nx;
        }
    }
    return tot;
}

template <bool MAX>
__global__ void __launch_bounds__(LG_TPB) k_scan_reduce(uint32_t* __restrict__ a, uint64_t n, uint32_t* __restrict__ part)
{
    for (uint64_t t = blockIdx.x; t * LG_TILE < n; t += gridDim.x)
    {
        const uint32_t tot = tile_scan<MAX, true>(a, t * LG_TILE, n, 0u, false);
        if (threadIdx.x == 0)
            part[t] = tot;
    }
}

// one workgroup: exclusive scan of the tile totals (in place)
template <bool MAX>
__global__ void __launch_bounds__(LG_TPB) k_scan_top(uint32_t* __restrict__ part, uint64_t nparts)
{
    uint32_t carry = 0;
    for (uint64_t b = 0; b < nparts; b += LG_TILE)
        carry = scan_op<MAX>(carry, tile_scan<MAX, true>(part, b, nparts, carry, true));
}

// exclusive sums (MAX = false: radix offsets) or inclusive maxima (MAX = true: run heads)
template <bool MAX>
__global__ void __launch_bounds__(LG_TPB) k_scan_apply(uint32_t* __restrict__ a, uint64_t n, const uint32_t* __restrict__ part)
{
    for (uint64_t t = blockIdx.x; t * LG_TILE < n; t += gridDim.x)
        tile_scan<MAX, !MAX>(a, t * LG_TILE, n, part[t], true);
}

// ---- stable LSD radix sort of (u64 key, u32 value) pairs ----
__global__ void __launch_bounds__(LG_TPB) k_rs_hist(const uint64_t* __restrict__ key, uint32_t n, uint32_t shift, uint32_t ntiles,
                                                    uint32_t* __restrict__ hist)
{
    __shared__ uint32_t h[256];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        h[threadIdx.x] = 0;
        __syncthreads();
        const uint64_t i0 = (uint64_t) t * LG_TILE;
        for (uint32_t k = 0; k < LG_PT; ++k)
        {
            const uint64_t i = i0 + (uint64_t) k * LG_TPB + threadIdx.x;
            if (i < n)
                atomicAdd(&h[(uint32_t) (key[i] >> shift) & 0xFFu], 1u);
        }
        __syncthreads();
        hist[(uint64_t) threadIdx.x * ntiles + t] = h[threadIdx.x];
        __syncthreads();
    }
}

// Lanes of the wave holding the same digit as this lane (8 ballots over the digit bits).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid)
{
    uint64_t m = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b)
    {
        const uint64_t x = __builtin_amdgcn_ballot_w64(valid && ((d >> b) & 1u));
        m &= ((d >> b) & 1u) ? x : ~x;
    }
    return valid ? m : 0ull;
}

__global__ void __launch_bounds__(LG_TPB) k_rs_scatter(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin, uint32_t n,
                                                       uint32_t shift, uint32_t ntiles, const uint32_t* __restrict__ off,
                                                       uint64_t* __restrict__ kout, uint32_t* __restrict__ vout)
{
    __shared__ uint32_t base[256];              // tile offset of each digit + elements of it already placed
    __shared__ uint32_t wcnt[LG_TPB / 64][256];  // this round: elements of each digit per wave
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        base[threadIdx.x] = off[(uint64_t) threadIdx.x * ntiles + t];
        for (uint32_t q = 0; q < LG_TPB / 64; ++q)
            wcnt[q][threadIdx.x] = 0;
        __syncthreads();
        const uint64_t i0 = (uint64_t) t * LG_TILE;
        for (uint32_t k = 0; k < LG_PT; ++k)
        {
            const uint64_t i     = i0 + (uint64_t) k * LG_TPB + threadIdx.x;
            const bool     valid = i < n;
            const uint64_t key   = valid ? kin[i] : 0ull;
            const uint32_t val   = valid ? vin[i] : 0u;
            const uint32_t d     = (uint32_t) (key >> shift) & 0xFFu;
            const uint64_t m     = match_digit(d, valid);
            const uint32_t below = (uint32_t) __popcll(m & ((1ull << lane) - 1ull));
            const bool     lead  = valid && below == 0;
            if (lead)
                wcnt[w][d] = (uint32_t) __popcll(m);
            __syncthreads();
            if (valid)
            {
                uint32_t pos = base[d] + below;
                for (uint32_t q = 0; q < w; ++q)
                    pos += wcnt[q][d];
                kout[pos] = key;
                vout[pos] = val;
            }
            __syncthreads();
            // advance the running counters by this round's counts, then clear them
            uint32_t add = 0;
            for (uint32_t q = 0; q < LG_TPB / 64; ++q)
            {
                add += wcnt[q][threadIdx.x];
                wcnt[q][threadIdx.x] = 0;
            }
            base[threadIdx.x] += add;
            __syncthreads();
        }
    }
}

template <typename T>
struct DevBuf
{
    T* p = nullptr;
    ~DevBuf() { (void) hipFree(p); }
    bool alloc(size_t n) { return hipMalloc((void**) &p, n * sizeof(T) + 16) == hipSuccess; }
};

template <bool MAX>
static bool scan_device(uint32_t* a, uint64_t n, uint32_t* part, hipStream_t s)
{
    const uint64_t nt   = (n + LG_TILE - 1) / LG_TILE;
    const dim3     grid((uint32_t) std::min<uint64_t>(nt, 65536));
    hipLaunchKernelGGL(k_scan_reduce<MAX>, grid, dim3(LG_TPB), 0, s, a, n, part);
    hipLaunchKernelGGL(k_scan_top<MAX>, dim3(1), dim3(LG_TPB), 0, s, part, nt);
    hipLaunchKernelGGL(k_scan_apply<MAX>, grid, dim3(LG_TPB), 0, s, a, n, (const uint32_t*) part);
    return hipGetLastError() == hipSuccess;
}

// Stable sort of (k0, v0) by the low `bits` key bits; the result is left in (k1, v1).
static bool radix_sort_pairs(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, uint32_t n, uint32_t bits, uint32_t* hist, uint32_t* part,
                             hipStream_t s)
{
    const uint32_t ntiles = (n + LG_TILE - 1) / LG_TILE;
    const dim3     grid(std::min<uint32_t>(ntiles, 65536));
    const uint32_t passes = (bits + 7) / 8;
    uint64_t*      ka[2]  = {k0, k1};
    uint32_t*      va[2]  = {v0, v1};
    // with an even number of passes, a first copy into (k1, v1) makes the last pass land there
    int cur = 0;
    if (passes % 2 == 0)
    {
        if (hipMemcpyAsync(k1, k0, (size_t) n * 8, hipMemcpyDeviceToDevice, s) != hipSuccess ||
            hipMemcpyAsync(v1, v0, (size_t) n * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return false;
        cur = 1;
    }
    for (uint32_t p = 0; p < passes; ++p)
    {
        hipLaunchKernelGGL(k_rs_hist, grid, dim3(LG_TPB), 0, s, ka[cur], n, 8 * p, ntiles, hist);
        if (!scan_device<false>(hist, 256ull * ntiles, part, s))
            return false;
        hipLaunchKernelGGL(k_rs_scatter, grid, dim3(LG_TPB), 0, s, ka[cur], va[cur], n, 8 * p, ntiles, hist, ka[cur ^ 1], va[cur ^ 1]);
        cur ^= 1;
    }
    return cur == 1 && hipGetLastError() == hipSuccess;
}

}  // namespace

bool bwt_encode_large(const uint8_t* d_in, uint32_t n, uint8_t* d_L, uint32_t* d_pi, hipStream_t s)
{
    if (n < 2)
    {
        if (n == 0)
            return false;
        return hipMemcpyAsync(d_L, d_in, 1, hipMemcpyDeviceToDevice, s) == hipSuccess && hipMemsetAsync(d_pi, 0, 4, s) == hipSuccess &&
               hipStreamSynchronize(s) == hipSuccess;
    }
    uint32_t B = 8;
    while (B < 32 && (1ull << B) < n)
        ++B;
    const uint64_t ntiles = ((uint64_t) n + LG_TILE - 1) / LG_TILE;
    const uint64_t nhist  = 256 * ntiles;
    DevBuf<uint64_t> k0, k1;
    DevBuf<uint32_t> i0, sa, rank, grp, flag, hist, part;
    if (!k0.alloc(n) || !k1.alloc(n) || !i0.alloc(n) || !sa.alloc(n) || !rank.alloc(n) || !grp.alloc(n) || !flag.alloc(1) || !hist.alloc(nhist) ||
        !part.alloc((std::max<uint64_t>(nhist, n) + LG_TILE - 1) / LG_TILE + 1))
    {
        bra_hip_report("bwt: large block of %u bytes: device allocation failed", n);
        return false;
    }
    const dim3 grid((uint32_t) std::min<uint64_t>(div_up(n, 256), 65536u)), tpb(256);
    for (uint64_t h = 0;; h = h ? 2 * h : 2)
    {
        // h = 0: the first two bytes; afterwards ranks cover h bytes and the key covers 2h
        if (h == 0)
            hipLaunchKernelGGL(k_lg_keys0, grid, tpb, 0, s, d_in, n, B, k0.p, i0.p);
        else
            hipLaunchKernelGGL(k_lg_keys, grid, tpb, 0, s, rank.p, n, (uint32_t) h, B, k0.p, i0.p);
        if (!radix_sort_pairs(k0.p, i0.p, k1.p, sa.p, n, 2 * B, hist.p, part.p, s))
            return false;
        const uint64_t covered = h ? 2 * h : 2;  // bytes of each rotation the sorted keys compare
        if (covered >= n)
            break;  // whole rotations compared: remaining ties are identical rotations (index order)
        if (hipMemsetAsync(flag.p, 0, 4, s) != hipSuccess)
            return false;
        hipLaunchKernelGGL(k_lg_heads, grid, tpb, 0, s, k1.p, n, grp.p, flag.p);
        if (!scan_device<true>(grp.p, n, part.p, s))
            return false;
        hipLaunchKernelGGL(k_lg_rank, grid, tpb, 0, s, sa.p, grp.p, n, rank.p);
        uint32_t tied = 0;
        if (hipMemcpyAsync(&tied, flag.p, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return false;
        if (!tied)
            break;  // every rotation's rank is final
    }
    hipLaunchKernelGGL(k_lg_emit, grid, tpb, 0, s, d_in, sa.p, n, d_L, d_pi);
    return hipStreamSynchronize(s) == hipSuccess && hipGetLastError() == hipSuccess;
}

}  // namespace bra
