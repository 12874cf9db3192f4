// ibwt.hip -- inverse BWT for a batch of independent blocks.
//
// Replaces bra_bwt_decode2 (reference src/encoders/bra_bwt.c:133-168): transform[first[c]+k] = the
// position of the k-th c in L (a stable partition of positions by byte, :141-159), then n steps
// `index = transform[index]; out[i] = L[index]` starting at the primary index (:161-167).
//
// The pointer chase is split with splitters: every S-th transform index plus the primary index.
// Main path (blocks < 2^24 bytes):
//   k_ib_hist / k_ib_scan / k_ib_scatter2 + 3  TL[k] = transform[k] | L[transform[k]] << 24, so one
//        4-byte load per step gives both the next index and the output byte;
//   k_ib_pair    TL2[k] = two steps from k in one 8-byte entry: T[T[k]], both output bytes and the
//        intermediate index T[k] (for the splitter test).  Its gathers are parallel and nearly
//        ordered (T is increasing inside every byte bucket, so the k of one bucket read TL at
//        increasing positions), unlike the walk's dependent loads, which it halves;
//   k_ib_walk3   persistent waves claim splitters from per-XCD queues (each XCD works through its
//        own range of blocks, so the random loads of an XCD stay in few blocks' TL2); a lane walks
//        from its splitter to the next one two steps per load, staging the bytes 16 at a time into
//        the splitter's slot (4 S bytes; longer hops continue in 256-byte chunks from a pool) and
//        records the hop;
//        lanes that finish claim the next splitter at once, so no lane idles on a long hop;
//   k_ib_chain3  one workgroup per block ranks the splitter list from the primary splitter by
//        pointer jumping in LDS -> output offset of every hop (and the primary cycle's length);
//   k_ib_copy16  sixteen lanes per hop stream its staged bytes to their output offset.
// A primary index on a cycle shorter than n (a periodic block) makes the output periodic with that
// cycle length, exactly like the reference (k_ib_repeat).  The round-1 two-walk kernels remain for
// blocks of >= 2^24 bytes, for callers that want the transform itself, and as the fallback when
// the overflow pool runs out.
#include "ibwt.h"
#include "prof.h"

#include <cstdlib>
#include <cstring>

namespace bra {

namespace {

constexpr int      TPB        = 256;
constexpr uint32_t MAX_SPLIT  = 4096;  // splitters per block (+1 for the primary index)
constexpr uint32_t ITILE      = 4096;

// main-path block record: splitter step S = 2^shift, ns regular splitters (0, S, 2S, ...) plus the
// primary index; the block's splitter slots (4 S bytes each) start at tslot in the slot buffer
struct IbBlk
{
    uint64_t off;
    uint64_t tslot;
    uint32_t len;
    uint32_t shift;
    uint32_t ns;
    uint32_t pad;
};
static_assert(sizeof(IbBlk) == 32, "IbBlk is stored in a uint64_t[4] per block");

__device__ __forceinline__ uint32_t split_step(uint32_t n)
{
    uint32_t s = 256;
    while ((n + s - 1) / s > MAX_SPLIT)
        s <<= 1;
    return s;
}

// per tile byte histogram of L
__global__ void __launch_bounds__(TPB) k_ib_hist(const uint8_t* __restrict__ L, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                 uint32_t* __restrict__ th, uint8_t* __restrict__ runny)
{
    // 16 consecutive bytes per thread, one LDS atomic per run of equal bytes (BWT output is
    // run-heavy: one atomic per byte made the lanes of a run serialise on one counter), 4 counter
    // copies by lane
    constexpr uint32_t HS = 256 + 16;
    __shared__ uint32_t h[4 * HS];
    const uint32_t      cp = (uint32_t) (lane_id() & 3) * HS;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            h[q * HS + threadIdx.x] = 0;
        __syncthreads();
        const Piece P = tiles[t];
        for (uint32_t i0 = threadIdx.x * 16; i0 < P.len; i0 += TPB * 16)
        {
            const uint8_t* src = L + P.off + i0;
            uint32_t       w[4] = {0, 0, 0, 0};
            const uint32_t n    = min(16u, P.len - i0);
            if (n == 16 && (((uintptr_t) src) & 15) == 0)
            {
                const uint4 v = *reinterpret_cast<const uint4*>(src);
                w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
            }
            else
                for (uint32_t j = 0; j < n; ++j)
                    w[j >> 2] |= (uint32_t) src[j] << (8 * (j & 3));
            uint32_t prev = w[0] & 0xFFu, run = 1;
            for (uint32_t j = 1; j < n; ++j)
            {
                const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                if (c == prev)
                    ++run;
                else
                {
                    atomicAdd(&h[cp + prev], run);
                    prev = c;
                    run  = 1;
                }
            }
            atomicAdd(&h[cp + prev], run);
        }
        __syncthreads();
        const uint32_t hv = h[threadIdx.x] + h[HS + threadIdx.x] + h[2 * HS + threadIdx.x] + h[3 * HS + threadIdx.x];
        th[(size_t) t * 256 + threadIdx.x] = hv;
        // k_ib_scatter2's tiles: few distinct bytes (a 64-position round then stores to few runs of
        // destinations: text, 16-symbol data); k_ib_scatter3's: many (uniform random data)
        const int distinct = __syncthreads_count(hv != 0);
        if (threadIdx.x == 0)
            runny[t] = distinct <= 48 ? 1 : 0;
        __syncthreads();
    }
}

// per block: tile offsets per byte = first[c] + sum over earlier tiles; *nopair counts the blocks
// that do not suit the two-step walk (k_ib_pair's gathers read TL at increasing positions inside a
// byte's bucket, 4 / frequency bytes apart: a byte rarer than 1/32 makes one 128-byte line per
// element, so a block where such bytes hold a quarter of the positions or more -- e.g. uniform
// random data -- is walked one step at a time, and with it the batch)
__global__ void __launch_bounds__(TPB) k_ib_scan(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count, uint32_t nblocks,
                                                 uint32_t* __restrict__ th, uint32_t* __restrict__ nopair)
{
    __shared__ uint32_t tmp[8];
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t t0 = first[b], nt = count[b], c = threadIdx.x;
        uint32_t       tot = 0, i = 0;
        // 16 tile rows in flight per round (one dependent load per tile made this a latency chain)
        for (; i + 16 <= nt; i += 16)
        {
            uint32_t h[16];
#pragma unroll
            for (int u = 0; u < 16; ++u)
                h[u] = th[(size_t) (t0 + i + u) * 256 + c];
#pragma unroll
            for (int u = 0; u < 16; ++u)
                tot += h[u];
        }
        for (; i < nt; ++i)
            tot += th[(size_t) (t0 + i) * 256 + c];
        uint32_t n;
        uint32_t run = block256_exclusive_sum(tot, tmp, &n);
        {
            uint32_t rare;
            __syncthreads();
            block256_exclusive_sum(32ull * tot <= n ? tot : 0u, tmp, &rare);
            if (c == 0 && nopair && 4ull * rare >= n)
                atomicAdd(nopair, 1u);
        }
        for (i = 0; i + 16 <= nt; i += 16)
        {
            uint32_t h[16];
#pragma unroll
            for (int u = 0; u < 16; ++u)
                h[u] = th[(size_t) (t0 + i + u) * 256 + c];
#pragma unroll
            for (int u = 0; u < 16; ++u)
            {
                th[(size_t) (t0 + i + u) * 256 + c] = run;
                run += h[u];
            }
        }
        for (; i < nt; ++i)
        {
            const size_t   o = (size_t) (t0 + i) * 256 + c;
            const uint32_t h = th[o];
            th[o]            = run;
            run += h;
        }
        __syncthreads();
    }
}

// stable scatter: T[off_c + rank of i among equal bytes before it in the tile] = i (block-local).
// One wave handles 64 consecutive positions at a time; ranks from 8 ballots per position.
__global__ void __launch_bounds__(64) k_ib_scatter(const uint8_t* __restrict__ L, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                   const uint32_t* __restrict__ th, const BlockDesc* __restrict__ blocks,
                                                   uint32_t* __restrict__ T)
{
    __shared__ uint32_t cnt[256];
    __shared__ uint4    tb4[ITILE / 16];  // the tile's bytes, loaded once (a byte load per step was a global round trip per 64 positions)
    const uint8_t*      tb   = reinterpret_cast<const uint8_t*>(tb4);
    const int           lane = lane_id();
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const Piece P = tiles[t];
        for (int i = lane; i < 256; i += 64)
            cnt[i] = th[(size_t) t * 256 + i];
        const uint8_t* src = L + P.off;
        if (P.len == ITILE && (((uintptr_t) src) & 15) == 0)
        {
#pragma unroll
            for (uint32_t q = 0; q < ITILE / 16 / 64; ++q)
                tb4[q * 64 + lane] = reinterpret_cast<const uint4*>(src)[q * 64 + lane];
        }
        else
            for (uint32_t i = lane; i < P.len; i += 64)
                reinterpret_cast<uint8_t*>(tb4)[i] = src[i];
        __syncthreads();
        const uint64_t boff = blocks[P.block].off;
        for (uint32_t base = 0; base < P.len; base += 64)
        {
            const uint32_t i     = base + lane;
            const bool     valid = i < P.len;
            const uint32_t c     = valid ? tb[i] : 0xFFFFFFFFu;
            uint64_t       m     = __ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 8; ++bit)
            {
                const uint64_t bb = __ballot(valid && ((c >> bit) & 1));
                m &= ((c >> bit) & 1) ? bb : ~bb;
            }
            const uint64_t lt   = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
            const uint32_t rank = (uint32_t) __popcll(m & lt);
            const uint32_t tot  = (uint32_t) __popcll(m);
            uint32_t       dst  = 0;
            if (valid)
                dst = cnt[c] + rank;
            __syncthreads();
            if (valid)
            {
                T[boff + dst] = P.start + i;
                // the last lane of each equal-byte group advances the counter
                if (rank == tot - 1)
                    cnt[c] += tot;
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ bool is_split(uint32_t y, uint32_t step, uint32_t pi) { return (y % step) == 0 || y == pi; }

// pass 1: each splitter walks to the next splitter
__global__ void k_ib_walk1(const BlockDesc* __restrict__ blocks, uint32_t nblocks, const uint32_t* __restrict__ pi,
                           const uint32_t* __restrict__ T, uint32_t* __restrict__ hop_next, uint32_t* __restrict__ hop_len)
{
    // grid.y = block, grid.x * blockDim.x >= splitters
    for (uint32_t b = blockIdx.y; b < nblocks; b += gridDim.y)
    {
        const BlockDesc B    = blocks[b];
        const uint32_t  step = split_step(B.len);
        const uint32_t  ns   = (B.len + step - 1) / step;  // regular splitters 0, step, 2*step, ...
        const uint32_t  p    = pi[b];
        for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k <= ns; k += gridDim.x * blockDim.x)
        {
            // k < ns: regular splitter k*step; k == ns: the primary index (if not regular)
            uint32_t s;
            if (k < ns)
                s = k * step;
            else
            {
                if (p % step == 0)
                    continue;
                s = p;
            }
            const uint32_t* Tb  = T + B.off;
            uint32_t        y   = s;
            uint32_t        len = 0;
            do
            {
                y = Tb[y];
                ++len;
            } while (!is_split(y, step, p) && len < B.len);
            const size_t o = (size_t) b * (MAX_SPLIT + 1) + k;
            hop_next[o]    = y;
            hop_len[o]     = len;
        }
    }
}

__device__ __forceinline__ uint32_t split_id(uint32_t y, uint32_t step, uint32_t ns, uint32_t p)
{
    return (y % step == 0) ? y / step : ns;  // y is a splitter
    (void) p;
}

// pass 2: one lane per block chains the hops starting at the primary index -> start offsets (in
// LDS); offsets of splitters not on the primary's cycle stay 0xFFFFFFFF.  cyc[b] = cycle length.
__global__ void __launch_bounds__(64) k_ib_chain(const BlockDesc* __restrict__ blocks, uint32_t nblocks, const uint32_t* __restrict__ pi,
                                                 const uint32_t* __restrict__ hop_next, const uint32_t* __restrict__ hop_len,
                                                 uint32_t* __restrict__ start, uint32_t* __restrict__ cyc)
{
    __shared__ uint32_t nx[MAX_SPLIT + 1], ln[MAX_SPLIT + 1], st[MAX_SPLIT + 1];
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const BlockDesc B    = blocks[b];
        const uint32_t  step = split_step(B.len);
        const uint32_t  ns   = (B.len + step - 1) / step;
        const uint32_t  p    = pi[b];
        const size_t    o    = (size_t) b * (MAX_SPLIT + 1);
        for (uint32_t k = lane_id(); k <= ns; k += 64)
        {
            st[k] = 0xFFFFFFFFu;
            nx[k] = split_id(hop_next[o + k], step, ns, p);
            ln[k] = hop_len[o + k];
        }
        __syncthreads();
        if (lane_id() == 0)
        {
            uint32_t k = split_id(p, step, ns, p);
            uint32_t t = 0;
            while (t < B.len && st[k] == 0xFFFFFFFFu)
            {
                st[k] = t;
                t += ln[k];
                k = nx[k];
            }
            cyc[b] = t < B.len ? t : B.len;
        }
        __syncthreads();
        for (uint32_t k = lane_id(); k <= ns; k += 64)
            start[o + k] = st[k];
        __syncthreads();
    }
}

// pass 3: re-walk and write out[start + j] = L[y]
__global__ void k_ib_walk2(const BlockDesc* __restrict__ blocks, uint32_t nblocks, const uint32_t* __restrict__ pi,
                           const uint32_t* __restrict__ T, const uint8_t* __restrict__ Lsrc, const uint32_t* __restrict__ start,
                           const uint32_t* __restrict__ hop_len, uint8_t* __restrict__ out)
{
    for (uint32_t b = blockIdx.y; b < nblocks; b += gridDim.y)
    {
        const BlockDesc B    = blocks[b];
        const uint32_t  step = split_step(B.len);
        const uint32_t  ns   = (B.len + step - 1) / step;
        const uint32_t  p    = pi[b];
        for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k <= ns; k += gridDim.x * blockDim.x)
        {
            const size_t   o  = (size_t) b * (MAX_SPLIT + 1) + k;
            const uint32_t st = start[o];
            if (st == 0xFFFFFFFFu)
                continue;
            const uint32_t  s   = (k < ns) ? k * step : p;
            const uint32_t* Tb  = T + B.off;
            const uint8_t*  Lb  = Lsrc + B.off;
            uint8_t*        ob  = out + B.off;
            const uint32_t  len = hop_len[o];
            uint32_t        y   = s;
            for (uint32_t j = 0; j < len && st + j < B.len; ++j)
            {
                y           = Tb[y];
                ob[st + j]  = Lb[y];
            }
        }
    }
}

// periodic primary cycle: out[i] = out[i mod c]
__global__ void k_ib_repeat(const BlockDesc* __restrict__ blocks, uint32_t nblocks, const uint32_t* __restrict__ cyc, uint8_t* __restrict__ out)
{
    for (uint32_t b = blockIdx.y; b < nblocks; b += gridDim.y)
    {
        const BlockDesc B = blocks[b];
        const uint32_t  c = cyc[b];
        if (c >= B.len || c == 0)
            continue;
        uint8_t* ob = out + B.off;
        for (uint32_t i = c + blockIdx.x * blockDim.x + threadIdx.x; i < B.len; i += gridDim.x * blockDim.x)
            ob[i] = ob[i % c];
    }
}

// ------------------------------------------------------------------------------------------------
// main path
// ------------------------------------------------------------------------------------------------
// stable scatter of (index | byte << 24): as k_ib_scatter, packed
__global__ void __launch_bounds__(64) k_ib_scatter2(const uint8_t* __restrict__ L, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                    const uint32_t* __restrict__ th, const BlockDesc* __restrict__ blocks,
                                                    uint32_t* __restrict__ TL, const uint8_t* __restrict__ runny)
{
    __shared__ uint32_t cnt[256];
    __shared__ uint4    tb4[ITILE / 16];  // the tile's bytes, loaded once (a byte load per step was a global round trip per 64 positions)
    const uint8_t*      tb   = reinterpret_cast<const uint8_t*>(tb4);
    const int           lane = lane_id();
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        if (!runny[t])
            continue;  // k_ib_scatter3's tile
        const Piece P = tiles[t];
        for (int i = lane; i < 256; i += 64)
            cnt[i] = th[(size_t) t * 256 + i];
        const uint8_t* src = L + P.off;
        if (P.len == ITILE && (((uintptr_t) src) & 15) == 0)
        {
#pragma unroll
            for (uint32_t q = 0; q < ITILE / 16 / 64; ++q)
                tb4[q * 64 + lane] = reinterpret_cast<const uint4*>(src)[q * 64 + lane];
        }
        else
            for (uint32_t i = lane; i < P.len; i += 64)
                reinterpret_cast<uint8_t*>(tb4)[i] = src[i];
        __syncthreads();
        const uint64_t boff = blocks[P.block].off;
        for (uint32_t base = 0; base < P.len; base += 64)
        {
            const uint32_t i     = base + lane;
            const bool     valid = i < P.len;
            const uint32_t c     = valid ? tb[i] : 0xFFFFFFFFu;
            uint64_t       m     = __ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 8; ++bit)
            {
                const uint64_t bb = __ballot(valid && ((c >> bit) & 1));
                m &= ((c >> bit) & 1) ? bb : ~bb;
            }
            const uint64_t lt   = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
            const uint32_t rank = (uint32_t) __popcll(m & lt);
            const uint32_t tot  = (uint32_t) __popcll(m);
            uint32_t       dst  = 0;
            if (valid)
                dst = cnt[c] + rank;
            __syncthreads();
            if (valid)
            {
                TL[boff + dst] = (P.start + i) | (c << 24);
                if (rank == tot - 1)
                    cnt[c] += tot;
            }
            __syncthreads();
        }
    }
}

// The same stable scatter staged through LDS: four waves per tile, wave w ranks positions
// [1024 w, 1024 w + 1024) among equal bytes (ballot match per 64 positions, a running count per
// byte and wave), the tile's entries are placed in LDS in their sorted order with their
// destinations beside them, and thread j stores the j-th of them: the stores of a workgroup run
// along the byte runs of the destination (k_ib_scatter2's store instructions hit up to 64
// destinations each).  For tiles of many distinct bytes (uniform random data); a tile of few
// distinct bytes (text, 16-symbol data: k_ib_hist's flag) stores to few runs of destinations per
// instruction already and stays with k_ib_scatter2, which is cheaper for it.
constexpr uint32_t IBS_WAVES = 4;
__global__ void __launch_bounds__(64 * IBS_WAVES) k_ib_scatter3(const uint8_t* __restrict__ L, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                               const uint32_t* __restrict__ th, const BlockDesc* __restrict__ blocks,
                                                               uint32_t* __restrict__ TL, const uint8_t* __restrict__ runny)
{
    constexpr uint32_t PER = ITILE / IBS_WAVES;  // positions per wave
    __shared__ uint4    tb4[ITILE / 16];
    __shared__ uint32_t wrun[IBS_WAVES][256];    // per wave and byte: count (then: offset among the tile's equal bytes)
    __shared__ uint32_t lstart[256];             // first sorted position of each byte in the tile
    __shared__ uint32_t gbase[256];              // block-local TL position of the tile's first entry of each byte
    __shared__ uint16_t rk[ITILE];               // rank among equal bytes before it in the wave's part
    __shared__ uint32_t sval[ITILE], sdst[ITILE];
    __shared__ uint32_t tmp[8];
    const uint8_t* tb   = reinterpret_cast<const uint8_t*>(tb4);
    const uint32_t lane = (uint32_t) lane_id(), w = wave_id();
    const uint64_t lt   = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        if (runny[t])
            continue;  // k_ib_scatter2's tile
        const Piece P = tiles[t];
        gbase[threadIdx.x] = th[(size_t) t * 256 + threadIdx.x];
#pragma unroll
        for (uint32_t v = 0; v < IBS_WAVES; ++v)
            wrun[v][threadIdx.x] = 0;
        const uint8_t* src = L + P.off;
        if (P.len == ITILE && (((uintptr_t) src) & 15) == 0)
            tb4[threadIdx.x] = reinterpret_cast<const uint4*>(src)[threadIdx.x];
        else
            for (uint32_t i = threadIdx.x; i < P.len; i += 64 * IBS_WAVES)
                reinterpret_cast<uint8_t*>(tb4)[i] = src[i];
        __syncthreads();
        // ranks inside the wave's part, counts per byte
        for (uint32_t r = 0; r < PER / 64; ++r)
        {
            const uint32_t i     = w * PER + r * 64 + lane;
            const bool     valid = i < P.len;
            const uint32_t c     = valid ? tb[i] : 0u;
            uint64_t       m     = __ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 8; ++bit)
            {
                const uint64_t bb = __ballot(valid && ((c >> bit) & 1));
                m &= ((c >> bit) & 1) ? bb : ~bb;
            }
            const uint32_t rank = (uint32_t) __popcll(m & lt), tot = (uint32_t) __popcll(m);
            uint32_t       before = 0;
            if (valid)
                before = wrun[w][c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (valid)
            {
                rk[i] = (uint16_t) (before + rank);
                if (rank == tot - 1)
                    wrun[w][c] = before + tot;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        __syncthreads();
        // per byte (thread c): the waves' offsets among the tile's equal bytes, the tile total and
        // the byte's first sorted position in the tile
        {
            const uint32_t c   = threadIdx.x;
            uint32_t       run = 0;
#pragma unroll
            for (uint32_t v = 0; v < IBS_WAVES; ++v)
            {
                const uint32_t n = wrun[v][c];
                wrun[v][c]       = run;
                run += n;
            }
            lstart[c] = block256_exclusive_sum(run, tmp);
        }
        __syncthreads();
        for (uint32_t r = 0; r < PER / 64; ++r)
        {
            const uint32_t i = w * PER + r * 64 + lane;
            if (i < P.len)
            {
                const uint32_t c = tb[i], k = wrun[w][c] + rk[i];
                sval[lstart[c] + k] = (P.start + i) | (c << 24);
                sdst[lstart[c] + k] = gbase[c] + k;
            }
        }
        __syncthreads();
        uint32_t* tl = TL + blocks[P.block].off;
        for (uint32_t j = threadIdx.x; j < P.len; j += 64 * IBS_WAVES)
            tl[sdst[j]] = sval[j];
        __syncthreads();
    }
}

// TL2[k] = T[T[k]] | L[T[k]] << 24 | L[T[T[k]]] << 32 | T[k] << 40 (block-local indices < 2^24):
// the byte of step 1, the byte of step 2, the index after step 2 and, for the splitter test, the
// index between them.  One workgroup per tile, tiles XCD-major (an XCD's gathers stay in its
// contiguous range of blocks), 16 positions per thread with all their gathers in flight.
__global__ void __launch_bounds__(TPB) k_ib_pair(const Piece* __restrict__ tiles, uint32_t ntiles, const BlockDesc* __restrict__ blocks,
                                                 const uint32_t* __restrict__ nopair, const uint32_t* __restrict__ TL, uint64_t* __restrict__ TL2)
{
    if (*nopair)
        return;  // the batch walks one step at a time
    constexpr int  PT = ITILE / TPB;
    const XcdTiles X  = xcd_tiles(ntiles);
    for (uint32_t t = X.t; t < X.end; t += X.step)
    {
        const Piece     P    = tiles[t];
        const uint32_t* tl   = TL + blocks[P.block].off;
        const uint64_t  o    = blocks[P.block].off + P.start;
        uint32_t        v1[PT], v2[PT];
#pragma unroll
        for (int j = 0; j < PT; ++j)
        {
            const uint32_t i = j * TPB + threadIdx.x;
            v1[j]            = i < P.len ? TL[o + i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < PT; ++j)
        {
            const uint32_t i = j * TPB + threadIdx.x;
            v2[j]            = i < P.len ? tl[v1[j] & 0xFFFFFFu] : 0u;
        }
#pragma unroll
        for (int j = 0; j < PT; ++j)
        {
            const uint32_t i = j * TPB + threadIdx.x;
            if (i < P.len)
                TL2[o + i] = (uint64_t) (v2[j] & 0xFFFFFFu) | ((uint64_t) (v1[j] >> 24) << 24) | ((uint64_t) (v2[j] >> 24) << 32) |
                             ((uint64_t) (v1[j] & 0xFFFFFFu) << 40);
        }
    }
}

// Hardware id (0-7) of the XCD the calling wave runs on (placement only: correctness never
// depends on it, every wave drains all eight queues).
__device__ __forceinline__ uint32_t xcd_id()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x & 7u;
}

struct WalkArgs
{
    const IbBlk*    blk;
    const uint32_t* pi;
    const uint32_t* cum;   // cum[b] = global id of block b's splitter 0 (cum[nblocks] = total)
    const uint32_t* xr;    // XCD x serves blocks [xr[x], xr[x+1])
    uint32_t*       qc;    // claim counters, one per XCD (32-word stride)
    const uint32_t* TL;
    const uint64_t* TL2;     // PAIR walks, unless *nopair
    const uint32_t* nopair;
    uint8_t*        slot;  // splitter slots
    uint8_t*        pool;  // overflow chunks of IB_CHUNK bytes
    uint32_t*       pool_ctr;
    uint32_t        pool_cap;
    uint32_t*       ovl_next;  // chunk -> next chunk of the same hop
    uint32_t*       hop_next;  // per splitter: block-local id of the next splitter
    uint32_t*       hop_len;
    uint32_t*       hop_ovf;   // first overflow chunk
};

constexpr uint32_t IB_CHUNK = 256;
// Persistent walk workgroups.  The grid sets how much of the TL arrays an XCD's lanes walk at once
// (each live lane works one splitter hop of S entries): the random loads hit those bytes, so the
// grid is sized to keep them near the XCD's 4 MB L2, with enough lanes left to hide the load
// latency.  256 x 1 MiB text (S = 64, scripts/gpu_r4v.sh): 256 WGs 3.55 ms, 384 3.07 (12 K lanes
// per XCD: 3 MB of TL), 512 3.18, 768 3.59, 1024 3.88, 2048 4.29, 4096 4.31; 32 x 8 MiB 16-symbol
// blocks (S = 512, scripts/gpu_r4aq.sh): 128 WGs 7.95 ms, 192 6.66, 256 6.49, 384 6.74.
__host__ inline uint32_t walk_grid(uint32_t max_shift)
{
    static const char* e = getenv("BRA_IB_WALKWG");  // measurement override
    if (e && *e)
        return (uint32_t) atoi(e);
    return max_shift <= 6 ? 384u : 256u;
}

// Walk two steps per load (k_ib_pair first) unless k_ib_scan counts a block that does not suit it?  Building TL2 writes 8
// bytes per element, more HBM time than the halved walk saves on blocks of up to 1 MiB (their TL
// fits an XCD's L2, so the one-step walk's loads hit it); BRA_IB_PAIR=0/1 overrides (measurement).
__host__ inline bool pair_walk(uint32_t max_shift)
{
    static const char* e = getenv("BRA_IB_PAIR");
    if (e && *e)
        return *e == '1';
    return max_shift > 6;
}

__device__ __forceinline__ uint8_t* walk_dst(const WalkArgs& a, uint8_t* slot, uint32_t cap, uint32_t o, uint32_t& chunk, uint32_t g)
{
    if (o < cap)
        return slot + o;
    const uint32_t r = o - cap;
    if ((r & (IB_CHUNK - 1)) == 0)
    {
        const uint32_t c = atomicAdd(a.pool_ctr, 1u);
        if (c >= a.pool_cap)
        {
            chunk = 0xFFFFFFFFu;
            return nullptr;  // pool exhausted: the host falls back to the two-walk path
        }
        if (r == 0)
            a.hop_ovf[g] = c;
        else if (chunk != 0xFFFFFFFFu)
            a.ovl_next[chunk] = c;
        chunk = c;
    }
    return chunk == 0xFFFFFFFFu ? nullptr : a.pool + (size_t) chunk * IB_CHUNK + (r & (IB_CHUNK - 1));
}

// WM_ONE: one step per load; WM_PAIR / WM_ONE_IF: two / one step per load if the batch suits /
// does not suit two-step walking (*nopair), else the kernel exits at once -- both are launched and
// one of them walks (a kernel holding both loops walked 9 % slower in pair mode).
enum WalkMode
{
    WM_ONE,
    WM_PAIR,
    WM_ONE_IF
};
template <int MODE>
__global__ void __launch_bounds__(256) k_ib_walk3(WalkArgs a)
{
    if (MODE != WM_ONE && (*a.nopair == 0) != (MODE == WM_PAIR))
        return;
    const int      lane = lane_id();
    const uint32_t x0   = xcd_id();
    uint32_t       t    = 0;  // queues tried: (x0 + t) & 7
    bool           act  = false;
    uint32_t       g = 0, k = 0, y = 0, j = 0, p = 0, mask = 0, shift = 0, ns = 0, cap = 0, chunk = 0xFFFFFFFFu;
    uint64_t       boff = 0, lo = 0, hi = 0;
    uint8_t*       slot = nullptr;
    while (true)
    {
        const uint64_t idle = __builtin_amdgcn_ballot_w64(!act);
        if (idle && t < 8)
        {
            const uint32_t n  = (uint32_t) __popcll(idle);
            const uint32_t x  = (x0 + t) & 7u;
            const uint32_t q0 = a.cum[a.xr[x]], q1 = a.cum[a.xr[x + 1]];
            uint32_t       b0 = 0;
            if (lane == 0)
                b0 = atomicAdd(&a.qc[x * 32], n);
            b0 = __builtin_amdgcn_readfirstlane(b0);
            if (b0 + n >= q1 - q0)
                ++t;
            if (!act)
            {
                const uint32_t pos = q0 + b0 + (uint32_t) __popcll(idle & ((1ull << lane) - 1ull));
                if (pos < q1)
                {
                    // block of splitter pos: last b in [xr[x], xr[x+1]) with cum[b] <= pos
                    uint32_t l = a.xr[x], h = a.xr[x + 1] - 1;
                    while (l < h)
                    {
                        const uint32_t mid = (l + h + 1) >> 1;
                        if (a.cum[mid] <= pos)
                            l = mid;
                        else
                            h = mid - 1;
                    }
                    const IbBlk B = a.blk[l];
                    g             = pos;
                    k             = pos - a.cum[l];
                    p             = a.pi[l];
                    shift         = B.shift;
                    mask          = (1u << shift) - 1u;
                    ns            = B.ns;
                    cap           = 4u << shift;
                    boff          = B.off;
                    slot          = a.slot + B.tslot + (size_t) k * cap;
                    chunk         = 0xFFFFFFFFu;
                    j             = 0;
                    lo = hi = 0;
                    if (k < ns)
                    {
                        y   = k << shift;
                        act = true;
                    }
                    else if (p & mask)
                    {
                        y   = p;
                        act = true;
                    }
                    else
                    {
                        a.hop_len[g]  = 0;  // the primary index is a regular splitter: no extra hop
                        a.hop_next[g] = 0xFFFFFFFFu;
                    }
                }
            }
        }
        if (!__builtin_amdgcn_ballot_w64(act))
        {
            if (t >= 8)
                break;
            continue;
        }
        if (act)
        {
            constexpr bool PAIR = MODE == WM_PAIR;
#pragma unroll 1
            for (int st = 0; st < (PAIR ? 16 : 32); ++st)
            {
                bool split;
                if constexpr (PAIR)
                {
                    // two steps per load; the hop ends at the intermediate index when that is a
                    // splitter (one byte), else after both (j stays even until then, so the 16-byte
                    // flushes fall on whole registers)
                    const uint64_t v  = a.TL2[boff + y];
                    const uint32_t y1 = (uint32_t) (v >> 40), y2 = (uint32_t) v & 0xFFFFFFu;
                    const uint64_t b1 = (v >> 24) & 0xFFu, b2 = (v >> 32) & 0xFFu;
                    const bool     s1 = (y1 & mask) == 0 || y1 == p;
                    if (s1)
                    {
                        lo = (lo >> 8) | (hi << 56);
                        hi = (hi >> 8) | (b1 << 56);
                        j += 1;
                        y = y1;
                    }
                    else
                    {
                        lo = (lo >> 16) | (hi << 48);
                        hi = (hi >> 16) | (b1 << 48) | (b2 << 56);
                        j += 2;
                        y = y2;
                    }
                    split = s1 || (y2 & mask) == 0 || y2 == p;
                }
                else
                {
                    const uint32_t v = a.TL[boff + y];
                    y                = v & 0xFFFFFFu;
                    lo               = (lo >> 8) | (hi << 56);
                    hi               = (hi >> 8) | ((uint64_t) (v >> 24) << 56);
                    ++j;
                    split = (y & mask) == 0 || y == p;
                }
                if ((j & 15) == 0 || split)
                {
                    const uint32_t nb = ((j - 1) & 15) + 1;  // staged bytes (the top nb of the register)
                    if (nb < 16)
                    {
                        const uint32_t sh = (16 - nb) * 8;  // move them to the bottom
                        if (sh >= 64)
                        {
                            lo = hi >> (sh - 64);
                            hi = 0;
                        }
                        else
                        {
                            lo = (lo >> sh) | (hi << (64 - sh));
                            hi >>= sh;
                        }
                    }
                    uint8_t* d = walk_dst(a, slot, cap, (j - 1) & ~15u, chunk, g);
                    if (d)
                        *reinterpret_cast<uint4*>(d) = make_uint4((uint32_t) lo, (uint32_t) (lo >> 32), (uint32_t) hi, (uint32_t) (hi >> 32));
                    lo = hi = 0;
                }
                if (split)
                {
                    a.hop_next[g] = (y == p && (p & mask)) ? ns : (y >> shift);
                    a.hop_len[g]  = j;
                    act           = false;
                    break;
                }
            }
        }
    }
}

// One workgroup per block: rank the splitter list from the primary splitter (pointer jumping in
// LDS over the hops), start offset of every hop on the primary cycle (0xFFFFFFFF elsewhere) and the
// cycle's length.
constexpr uint32_t IB_MAXS   = 16385;  // splitters per block (16384 regular + the primary index)
constexpr uint32_t IB_CH_TPB = 1024;

__global__ void __launch_bounds__(IB_CH_TPB) k_ib_chain3(const IbBlk* __restrict__ blk, const uint32_t* __restrict__ pi,
                                                         const uint32_t* __restrict__ cum, uint32_t nblocks,
                                                         const uint32_t* __restrict__ hop_next, const uint32_t* __restrict__ hop_len,
                                                         uint32_t* __restrict__ start, uint32_t* __restrict__ cyc, uint32_t* __restrict__ order,
                                                         uint32_t* __restrict__ cnt)
{
    __shared__ uint16_t nx[IB_MAXS];
    __shared__ uint32_t R[IB_MAXS];
    __shared__ uint16_t C[IB_MAXS];  // hops from q to the end of the chain (its rank from the end)
    __shared__ uint32_t sh_tot;
    constexpr uint16_t  END = 0xFFFF;
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const IbBlk    B    = blk[b];
        const uint32_t base = cum[b], nn = cum[b + 1] - base;
        const uint32_t p = pi[b], mask = (1u << B.shift) - 1u;
        const uint32_t s0 = (p & mask) ? B.ns : (p >> B.shift);
        for (uint32_t q = threadIdx.x; q < nn; q += IB_CH_TPB)
        {
            const uint32_t h = hop_next[base + q];
            nx[q]            = h == 0xFFFFFFFFu ? END : (uint16_t) h;
            R[q]             = hop_len[base + q];
            C[q]             = R[q] ? 1 : 0;  // hops that produce output (unused splitter slots have none)
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nn; q += IB_CH_TPB)
            if (nx[q] == s0)
                nx[q] = END;  // the cycle through s0 ends before s0
        __syncthreads();
        uint32_t rounds = 1;
        while ((1u << rounds) < nn)
            ++rounds;
        for (uint32_t r = 0; r <= rounds; ++r)
        {
            uint32_t nn2[(IB_MAXS + IB_CH_TPB - 1) / IB_CH_TPB], rr[(IB_MAXS + IB_CH_TPB - 1) / IB_CH_TPB], cc[(IB_MAXS + IB_CH_TPB - 1) / IB_CH_TPB];
#pragma unroll
            for (uint32_t u = 0; u < (IB_MAXS + IB_CH_TPB - 1) / IB_CH_TPB; ++u)
            {
                const uint32_t q = threadIdx.x + u * IB_CH_TPB;
                nn2[u]           = END;
                rr[u]            = 0;
                cc[u]            = 0;
                if (q < nn && nx[q] != END)
                {
                    nn2[u] = nx[nx[q]];
                    rr[u]  = R[nx[q]];
                    cc[u]  = C[nx[q]];
                }
            }
            __syncthreads();
#pragma unroll
            for (uint32_t u = 0; u < (IB_MAXS + IB_CH_TPB - 1) / IB_CH_TPB; ++u)
            {
                const uint32_t q = threadIdx.x + u * IB_CH_TPB;
                if (q < nn && nx[q] != END)
                {
                    nx[q] = (uint16_t) nn2[u];
                    R[q] += rr[u];
                    C[q] = (uint16_t) (C[q] + cc[u]);
                }
            }
            __syncthreads();
        }
        if (threadIdx.x == 0)
        {
            sh_tot = R[s0];
            cyc[b] = min(R[s0], B.len);
            cnt[b] = C[s0];
        }
        __syncthreads();
        const uint32_t tot = sh_tot, ctot = C[s0];
        for (uint32_t q = threadIdx.x; q < nn; q += IB_CH_TPB)
        {
            start[base + q] = (nx[q] == END && hop_len[base + q] != 0) ? tot - R[q] : 0xFFFFFFFFu;
            if (nx[q] == END && hop_len[base + q] != 0 && C[q] <= ctot)
                order[base + ctot - C[q]] = q;  // the chain's hops in output order
        }
        __syncthreads();
    }
}

// Sixteen lanes per hop, four hops per wave: lane l copies source bytes 16 l, 16 l + 256, ... of
// its hop's slot to the output with unaligned 16-byte stores, so one store instruction writes four
// contiguous stretches (the round-4 lane-per-hop copy stored 4 bytes to each of 64 lines per
// instruction: bound by the L2 request rate, not by bytes).  The first 256 bytes of 8 hops are
// loaded before any of them is stored (a hop-by-hop loop left every hop's load latency exposed:
// 0.50 -> 0.28 ms on 256 x 1 MiB text); a hop's partial last 16 bytes go out as at most four
// narrower stores (the next hop owns the bytes after it).
typedef uint32_t __attribute__((aligned(1))) u32_u;
typedef uint4 __attribute__((aligned(1))) u128_u;
typedef uint64_t __attribute__((aligned(1))) u64_u;
typedef uint16_t __attribute__((aligned(1))) u16_u;
constexpr uint32_t CP_BATCH = 8;

// the first k (1..16) bytes of v to dst (unaligned): one 16-byte store, or at most four narrower
// ones for the partial tail of a hop (the bytes after it belong to the next hop)
__device__ __forceinline__ void store_head(uint8_t* dst, uint4 v, uint32_t k)
{
    if (k == 16)
    {
        *reinterpret_cast<u128_u*>(dst) = v;
        return;
    }
    uint32_t w0 = v.x, w1 = v.y, w2 = v.z;
    if (k & 8)
    {
        *reinterpret_cast<u64_u*>(dst) = (uint64_t) w0 | (uint64_t) w1 << 32;
        dst += 8, w0 = w2, w1 = v.w;
    }
    if (k & 4)
    {
        *reinterpret_cast<u32_u*>(dst) = w0;
        dst += 4, w0 = w1;
    }
    if (k & 2)
    {
        *reinterpret_cast<u16_u*>(dst) = (uint16_t) w0;
        dst += 2, w0 >>= 16;
    }
    if (k & 1)
        *dst = (uint8_t) w0;
}

__global__ void __launch_bounds__(256) k_ib_copy16(const IbBlk* __restrict__ blk, const uint32_t* __restrict__ cum, const uint32_t* __restrict__ cnt,
                                                   const uint32_t* __restrict__ order, uint32_t nblocks,
                                                   const uint32_t* __restrict__ start, const uint32_t* __restrict__ hop_len,
                                                   const uint32_t* __restrict__ hop_ovf, const uint32_t* __restrict__ ovl_next,
                                                   const uint8_t* __restrict__ slots, const uint8_t* __restrict__ pool, uint32_t pool_cap,
                                                   uint8_t* __restrict__ out)
{
    const uint32_t lane = (uint32_t) lane_id(), l = lane & 15u, g0 = lane & ~15u;  // g0: the group's first lane
    for (uint32_t b = blockIdx.y; b < nblocks; b += gridDim.y)
    {
        const IbBlk    B    = blk[b];
        const uint32_t base = cum[b], nn = cum[b + 1] - base, cap = 4u << B.shift;
        uint8_t*       ob   = out + B.off;
        const uint32_t nh   = min(cnt[b], nn);
        // a group takes 16 consecutive hops in output order at a time: lane l loads hop l's record
        // (two dependent round trips for 16 hops, not per hop), then the group copies the 16 hops
        // one after the other (they are adjacent in the output)
        for (uint32_t r0 = ((blockIdx.x * blockDim.x + threadIdx.x) >> 4) * 16; r0 < nh; r0 += ((gridDim.x * blockDim.x) >> 4) * 16)
        {
            const uint32_t r   = r0 + l;
            uint32_t       q   = 0, st = 0xFFFFFFFFu, len = 0;
            if (r < nh)
            {
                q  = order[base + r];
                st = start[base + q];
                if (st < B.len)
                    len = min(hop_len[base + q], B.len - st);
            }
            for (uint32_t h0 = 0; h0 < 16; h0 += CP_BATCH)
            {
                // the first 256 bytes of CP_BATCH hops (a whole slot when S = 64): all loads in
                // flight before the first store
                uint4 v[CP_BATCH];
#pragma unroll
                for (uint32_t i = 0; i < CP_BATCH; ++i)
                {
                    const uint32_t hq = (uint32_t) __shfl((int) q, (int) (g0 + h0 + i), 64);
                    const uint32_t hl = (uint32_t) __shfl((int) len, (int) (g0 + h0 + i), 64);
                    v[i]              = make_uint4(0, 0, 0, 0);
                    if (16 * l < min(hl, cap))
                        v[i] = reinterpret_cast<const uint4*>(slots + B.tslot + (size_t) hq * cap)[l];
                }
#pragma unroll
                for (uint32_t i = 0; i < CP_BATCH; ++i)
                {
                    const uint32_t hs = (uint32_t) __shfl((int) st, (int) (g0 + h0 + i), 64);
                    const uint32_t hl = (uint32_t) __shfl((int) len, (int) (g0 + h0 + i), 64);
                    const uint32_t m  = min(hl, cap), o = 16 * l;
                    if (hs < B.len && o < m)
                        store_head(ob + hs + o, v[i], min(m - o, 16u));
                }
            }
            for (uint32_t h = 0; h < 16; ++h)
            {
                const uint32_t hq = (uint32_t) __shfl((int) q, (int) (g0 + h), 64);
                const uint32_t hs = (uint32_t) __shfl((int) st, (int) (g0 + h), 64);
                const uint32_t hl = (uint32_t) __shfl((int) len, (int) (g0 + h), 64);
                if (hs >= B.len || hl <= 256)
                    continue;
                // the rest of a slot of more than 256 bytes (S > 64), then the overflow chunks
                const uint8_t* src = slots + B.tslot + (size_t) hq * cap;
                const uint32_t m   = min(hl, cap);
                uint8_t*       dst = ob + hs;
                for (uint32_t o = 256 + 16 * l; o < m; o += 256)
                    store_head(dst + o, *reinterpret_cast<const uint4*>(src + o), min(m - o, 16u));
                uint32_t c = hl > cap ? hop_ovf[base + hq] : 0xFFFFFFFFu;
                for (uint32_t o0 = cap; o0 < hl && c < pool_cap; o0 += IB_CHUNK)
                {
                    const uint8_t* cs = pool + (size_t) c * IB_CHUNK;
                    const uint32_t mm = min(IB_CHUNK, hl - o0);
                    for (uint32_t o = 16 * l; o < mm; o += 256)
                    {
                        store_head(dst + o0 + o, *reinterpret_cast<const uint4*>(cs + o), min(mm - o, 16u));
                    }
                    c = ovl_next[c];
                }
            }
        }
    }
}

}  // namespace

bool IbwtWorkspace::reserve(uint64_t n, uint32_t nblocks, uint32_t ntiles)
{
    if (n > cap_n)
    {
        cap_n            = 0;
        const uint64_t c = n + n / 8 + 4096;
        if (!dev_alloc(T, c))
            return false;
        cap_n = c;
    }
    if (ntiles > cap_t)
    {
        cap_t            = 0;
        const uint32_t c = ntiles + ntiles / 4 + 64;
        if (!dev_alloc(th, (uint64_t) c * 256 + c / 4 + 1))  // + one byte per tile (k_ib_hist's run flag)
            return false;
        cap_t = c;
    }
    if (nblocks > cap_b)
    {
        cap_b            = 0;
        const uint32_t c = nblocks + 8;
        if (!dev_alloc(hop_next, (uint64_t) c * (MAX_SPLIT + 1)) || !dev_alloc(hop_len, (uint64_t) c * (MAX_SPLIT + 1)) ||
            !dev_alloc(start, (uint64_t) c * (MAX_SPLIT + 1)) || !dev_alloc(cyc, c) || (!nopair && !dev_alloc(nopair, 1)))
            return false;
        cap_b = c;
    }
    return true;
}

void IbwtWorkspace::release()
{
    tiling.release();
    (void) hipFree(T);
    (void) hipFree(T2);
    (void) hipFree(th);
    (void) hipFree(hop_next);
    (void) hipFree(hop_len);
    (void) hipFree(start);
    (void) hipFree(cyc);
    (void) hipFree(nopair);
    for (void* p : {(void*) blk, (void*) cum, (void*) ctl, (void*) m_next, (void*) m_len, (void*) m_ovf, (void*) m_start, (void*) ovl_next,
                    (void*) slot, (void*) pool, (void*) m_order, (void*) m_cnt})
        (void) hipFree(p);
    *this = IbwtWorkspace{};
}

// the round-1 path: two walks over the transform (T and L separate)
static bool ibwt_two_walk(IbwtWorkspace& w, const uint8_t* d_L, const uint32_t* d_pi, const BlockDesc* d_blocks, uint32_t nblocks,
                          uint8_t* d_out, hipStream_t s)
{
    const uint32_t nt = w.tiling.n;
    hipLaunchKernelGGL(k_ib_scatter, dim3(std::min<uint32_t>(nt, 16384)), dim3(64), 0, s, d_L, w.tiling.d_pieces, nt, w.th, d_blocks, w.T);
    const dim3 g(div_up(MAX_SPLIT + 1, 128), std::min<uint32_t>(nblocks, 65535));
    hipLaunchKernelGGL(k_ib_walk1, g, dim3(128), 0, s, d_blocks, nblocks, d_pi, w.T, w.hop_next, w.hop_len);
    hipLaunchKernelGGL(k_ib_chain, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(64), 0, s, d_blocks, nblocks, d_pi, w.hop_next, w.hop_len,
                       w.start, w.cyc);
    hipLaunchKernelGGL(k_ib_walk2, g, dim3(128), 0, s, d_blocks, nblocks, d_pi, w.T, d_L, w.start, w.hop_len, d_out);
    hipLaunchKernelGGL(k_ib_repeat, dim3(64, std::min<uint32_t>(nblocks, 65535)), dim3(256), 0, s, d_blocks, nblocks, w.cyc, d_out);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

bool IbwtWorkspace::reserve_main(uint32_t nblocks, uint32_t nsplit, uint64_t slot_bytes)
{
    if (nblocks + 1 > cap_mb)
    {
        cap_mb           = 0;
        const uint32_t c = nblocks + 64;
        if (!dev_alloc(blk, (uint64_t) c * 4) || !dev_alloc(cum, c) || !dev_alloc(ctl, 512) || !dev_alloc(m_cnt, c))
            return false;
        cap_mb = c;
    }
    if (nsplit > cap_ms)
    {
        cap_ms           = 0;
        const uint32_t c = nsplit + nsplit / 8 + 64;
        const uint32_t pc = c / 8 + 256;  // overflow chunks (hops longer than 4 S: ~2 % of them)
        if (!dev_alloc(m_next, c) || !dev_alloc(m_len, c) || !dev_alloc(m_ovf, c) || !dev_alloc(m_start, c) || !dev_alloc(m_order, c) ||
            !dev_alloc(ovl_next, pc) ||
            !dev_alloc(pool, (uint64_t) pc * IB_CHUNK))
            return false;
        cap_ms   = c;
        pool_cap = pc;
    }
    if (slot_bytes > cap_slot)
    {
        cap_slot         = 0;
        const uint64_t c = slot_bytes + slot_bytes / 8 + 4096;
        if (!dev_alloc(slot, c))
            return false;
        cap_slot = c;
    }
    return true;
}

bool ibwt_device(IbwtWorkspace& w, const uint8_t* d_L, const uint32_t* d_pi, const BlockDesc* d_blocks, const BlockDesc* h_blocks,
                 uint32_t nblocks, uint8_t* d_out, hipStream_t s, bool keep_transform)
{
    if (!w.tiling.build(h_blocks, nblocks, ITILE, s))
        return false;
    uint64_t N = 0;
    bool     main_path = !keep_transform;
    for (uint32_t b = 0; b < nblocks; ++b)
    {
        N = std::max<uint64_t>(N, h_blocks[b].off + h_blocks[b].len);
        main_path = main_path && h_blocks[b].len < (1u << 24);
    }
    const uint32_t nt = w.tiling.n;
    if (!w.reserve(N, nblocks, nt))
        return false;
    uint8_t* runny = reinterpret_cast<uint8_t*>(w.th + (size_t) w.cap_t * 256);  // per tile: k_ib_scatter2 (1) or k_ib_scatter3 (0)
    hipLaunchKernelGGL(k_ib_hist, dim3(std::min<uint32_t>(nt, 8192)), dim3(TPB), 0, s, d_L, w.tiling.d_pieces, nt, w.th, runny);
    BRA_HIP_CHECK(hipMemsetAsync(w.nopair, 0, 4, s));
    hipLaunchKernelGGL(k_ib_scan, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(TPB), 0, s, w.tiling.d_first, w.tiling.d_count, nblocks, w.th,
                       w.nopair);
    if (!main_path)
        return ibwt_two_walk(w, d_L, d_pi, d_blocks, nblocks, d_out, s);

    // splitter geometry: step S >= 64, at most 16384 regular splitters per block; slots of 4 S bytes
    if (w.h_key.size() != nblocks || !std::equal(w.h_key.begin(), w.h_key.end(), h_blocks,
                                                 [](const BlockDesc& a, const BlockDesc& b) { return a.off == b.off && a.len == b.len; }))
    {
        w.h_blk.assign(nblocks * 4, 0);
        std::vector<uint32_t> cum(nblocks + 1), ctl(512, 0);
        uint64_t              slot = 0;
        uint32_t              G = 0, max_shift = 6;
        for (uint32_t b = 0; b < nblocks; ++b)
        {
            const uint32_t n     = h_blocks[b].len;
            uint32_t       shift = 6;
            while (((uint64_t) n + (1u << shift) - 1) >> shift > IB_MAXS - 1)
                ++shift;
            max_shift = std::max(max_shift, shift);
            const uint32_t ns = (uint32_t) (((uint64_t) n + (1u << shift) - 1) >> shift);
            IbBlk          B{h_blocks[b].off, slot, n, shift, ns, 0};
            std::memcpy(&w.h_blk[(size_t) b * 4], &B, sizeof B);
            cum[b] = G;
            G += ns + 1;
            slot += (uint64_t) (ns + 1) * (4u << shift);
        }
        cum[nblocks] = G;
        w.walk_wg    = walk_grid(max_shift);
        w.pair       = pair_walk(max_shift);
        // XCD x serves blocks [xr[x], xr[x+1]): contiguous eighths of the batch
        for (uint32_t x = 0; x <= 8; ++x)
            ctl[256 + x] = (uint32_t) ((uint64_t) nblocks * x / 8);
        if (!w.reserve_main(nblocks, G, slot))
            return false;
        if (w.pair && N > w.cap_n2)
        {
            w.cap_n2 = 0;
            if (!dev_alloc(w.T2, N + N / 8 + 4096))
                return false;
            w.cap_n2 = N + N / 8 + 4096;
        }
        w.G = G;
        w.h_key.clear();
        BRA_HIP_CHECK(hipMemcpyAsync(w.blk, w.h_blk.data(), (size_t) nblocks * sizeof(IbBlk), hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipMemcpyAsync(w.cum, cum.data(), (size_t) (nblocks + 1) * 4, hipMemcpyHostToDevice, s));
        w.h_ctl = ctl;
        BRA_HIP_CHECK(hipMemcpyAsync(w.ctl, w.h_ctl.data(), 512 * 4, hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipStreamSynchronize(s));  // host vectors are the copies' sources
        w.h_key.assign(h_blocks, h_blocks + nblocks);
    }
    const IbBlk* blk = reinterpret_cast<const IbBlk*>(w.blk);
    // ctl[0..255]: 8 claim counters (32-word stride), ctl[256..264]: XCD block ranges, ctl[300]: pool counter
    BRA_HIP_CHECK(hipMemsetAsync(w.ctl, 0, 256 * 4, s));
    BRA_HIP_CHECK(hipMemsetAsync(w.ctl + 300, 0, 4, s));
    hipLaunchKernelGGL(k_ib_scatter2, dim3(std::min<uint32_t>(nt, 16384)), dim3(64), 0, s, d_L, w.tiling.d_pieces, nt, w.th, d_blocks, w.T, runny);
    // (about the resident capacity: 50 KiB of LDS per workgroup, 3 per CU; on text every tile is
    // k_ib_scatter2's and this launch only reads the flags)
    hipLaunchKernelGGL(k_ib_scatter3, dim3(std::min<uint32_t>(nt, 1024)), dim3(64 * IBS_WAVES), 0, s, d_L, w.tiling.d_pieces, nt, w.th, d_blocks,
                       w.T, runny);
    if (w.pair)
    {
        BRA_PROF(P_DEC_IB_PAIR, s);
        hipLaunchKernelGGL(k_ib_pair, dim3(xcd_grid(std::min<uint32_t>(nt, 8192))), dim3(TPB), 0, s, w.tiling.d_pieces, nt, d_blocks, w.nopair, w.T,
                           w.T2);
    }
    WalkArgs a{blk, d_pi, w.cum, w.ctl + 256, w.ctl, w.T, w.T2, w.nopair, w.slot, w.pool, w.ctl + 300, w.pool_cap, w.ovl_next, w.m_next, w.m_len, w.m_ovf};
    {
        BRA_PROF(P_DEC_IB_WALK, s);
        if (g_prof)
        {
            double n = 0;  // algorithmic bytes per element: one output byte and a 4-byte TL entry (PAIR: half an 8-byte TL2 entry)
            for (uint32_t b = 0; b < nblocks; ++b)
                n += h_blocks[b].len;
            prof_bytes(P_DEC_IB_WALK, 5.0 * n);
            prof_bytes(P_DEC_IB_PAIR, 16.0 * n);  // TL read twice, TL2 written
        }
        if (w.pair)
        {
            hipLaunchKernelGGL(k_ib_walk3<WM_PAIR>, dim3(w.walk_wg), dim3(256), 0, s, a);
            hipLaunchKernelGGL(k_ib_walk3<WM_ONE_IF>, dim3(w.walk_wg), dim3(256), 0, s, a);
        }
        else
            hipLaunchKernelGGL(k_ib_walk3<WM_ONE>, dim3(w.walk_wg), dim3(256), 0, s, a);
    }
    hipLaunchKernelGGL(k_ib_chain3, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(IB_CH_TPB), 0, s, blk, d_pi, w.cum, nblocks, w.m_next,
                       w.m_len, w.m_start, w.cyc, w.m_order, w.m_cnt);
    hipLaunchKernelGGL(k_ib_copy16, dim3(64, std::min<uint32_t>(nblocks, 65535)), dim3(256), 0, s, blk, w.cum, w.m_cnt, w.m_order, nblocks, w.m_start,
                       w.m_len, w.m_ovf, w.ovl_next, w.slot, w.pool, w.pool_cap, d_out);
    hipLaunchKernelGGL(k_ib_repeat, dim3(64, std::min<uint32_t>(nblocks, 65535)), dim3(256), 0, s, d_blocks, nblocks, w.cyc, d_out);
    BRA_HIP_CHECK(hipGetLastError());
    // overflow pool exhausted (hops far longer than 4 S, e.g. adversarial inputs): redo the batch
    // with the two-walk path, which needs no staging
    uint32_t used = 0;
    BRA_HIP_CHECK(hipMemcpyAsync(&used, w.ctl + 300, 4, hipMemcpyDeviceToHost, s));
    BRA_HIP_CHECK(hipStreamSynchronize(s));
    if (used > w.pool_cap)
        return ibwt_two_walk(w, d_L, d_pi, d_blocks, nblocks, d_out, s);
    return true;
}

}  // namespace bra
