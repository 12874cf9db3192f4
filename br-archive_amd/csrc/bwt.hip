// bwt.hip -- Burrows-Wheeler transform of cyclic rotations for a batch of independent blocks.
//
// Replaces bra_bwt_encode2 (reference src/encoders/bra_bwt.c:73-108: qsort_r of rotation indices
// with the cyclic byte comparator of :31-53, then L[j] = buf[(SA[j]+n-1) % n], pi = j with SA[j]==0).
// Parity contract: L is tie-order independent (equal rotations have
// equal last bytes); pi = number of rotations strictly smaller than rotation 0, i.e. the start
// of rotation 0's group of identical rotations (glibc qsort_r is a stable merge sort).
//
// Algorithm (all blocks of the batch at once; every kernel is grid-strided over a work list):
//   level 0      bucket every position of every block by its first byte (tile histograms in LDS,
//                per-block scan, LDS-staged scatter).  Each element carries an 8-byte key (the
//                rotation's bytes [kd, kd+8), big-endian) and a payload (prev byte << 24 | index).
//   level >= 1   MSD radix passes on the next key byte for buckets larger than JOB_MAX, with the
//                key re-gathered from the input every 8 bytes.  Sub-buckets of <= JOB_MAX elements
//                are packed into wave jobs.
//   wave jobs    one wave sorts <= 256 elements in registers (bitonic, 4 per lane), then refines
//                groups of equal keys by gathering 7 more bytes per round (group id in the top 8
//                bits keeps groups in place) until no ties remain, the depth reaches n (ties are
//                then identical rotations), or a depth cap sends the group to the fallback.
//   fallback     Larsson-Sadakane style prefix doubling on ranks for the groups still tied (only
//                pathological, highly repetitive blocks get here), using the same MSD/wave
//                machinery on 32-bit rank keys.
#include "bwt.h"
#include "prof.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace bra {

namespace {

constexpr int      TILE         = 4096;  // elements per tile (256 threads x 16)
constexpr int      TPB          = 256;
constexpr int      PER_THREAD   = TILE / TPB;
constexpr uint32_t JOB_MAX      = 256;  // elements one wave sorts in registers
constexpr uint32_t DCAP_BIG     = 64;   // MSD depth after which a big bucket goes to the fallback
constexpr uint32_t DCAP_JOB     = 512;  // refinement depth after which a tied group goes to the fallback
constexpr uint32_t RANK_KEYBYTES = 4;   // rank keys are 32-bit

enum : uint32_t { MODE_STRING = 0, MODE_RANK = 1 };

struct Bucket
{
    uint32_t start;   // global slot of the first element
    uint32_t len;
    uint32_t d;       // MSD depth (STRING: bytes shared; RANK: key bytes consumed)
    uint32_t kd;      // key base depth (bytes [kd, kd+8) are in the key)
    uint32_t block;
    uint32_t buf;     // which KV buffer holds the elements
    uint32_t gdepth;  // RANK mode: string depth of the group
    uint32_t tile0;   // first tile of this bucket at the current level
};

struct Job
{
    uint32_t start, len, kd, buf, block, gdepth;
};

struct Group
{
    uint32_t start, len, depth, block;
};

struct Counters
{
    uint32_t n_big;       // buckets appended to the next level
    uint32_t n_jobs;
    uint32_t n_groups;    // fallback groups appended (next round)
    uint32_t n_tiles;     // tiles of the current level
    uint32_t overflow;    // a work list overflowed (fatal)
    uint32_t g_members;   // members of appended fallback groups
    uint32_t hmin;        // min depth of appended fallback groups
    uint32_t n_elems;     // elements in this level's big buckets (k_build_tiles)
    uint32_t n_moved;     // elements the level's scatter moves (k_scan)
    uint32_t pad[3];
};

// -------------------------------------------------------------------------------------------------
// level 0: byte histograms of input tiles
// -------------------------------------------------------------------------------------------------
struct L0Tile
{
    uint32_t block, start;
};

__global__ void __launch_bounds__(TPB) k_l0_hist(const uint8_t* __restrict__ in, const BlockDesc* __restrict__ blocks,
                                                 const L0Tile* __restrict__ tiles, uint32_t ntiles, uint32_t* __restrict__ tile_hist)
{
    __shared__ uint32_t h[256];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        h[threadIdx.x] = 0;
        __syncthreads();
        const L0Tile    T   = tiles[t];
        const BlockDesc B   = blocks[T.block];
        const uint32_t  cnt = min((uint32_t) TILE, B.len - T.start);
        const uint8_t*  p   = in + B.off + T.start;
        for (uint32_t i = threadIdx.x; i < cnt; i += TPB)
            atomicAdd(&h[p[i]], 1u);
        __syncthreads();
        tile_hist[(size_t) t * 256 + threadIdx.x] = h[threadIdx.x];
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------------------
// level >= 1: histogram of the next key byte (re-gathering the key every 8 bytes)
// -------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t eff_kd(const Bucket& B, uint32_t mode)
{
    return (mode == MODE_STRING && B.d - B.kd >= 8) ? B.d : B.kd;
}

__device__ __forceinline__ uint32_t key_digit(uint64_t key, uint32_t d, uint32_t kd)
{
    return (uint32_t) (key >> (56 - 8 * (d - kd))) & 0xFFu;
}

template <uint32_t MODE>
__global__ void __launch_bounds__(TPB) k_hist(const uint8_t* __restrict__ in, const BlockDesc* __restrict__ blocks,
                                              const Bucket* __restrict__ buckets, const uint32_t* __restrict__ tile_bucket,
                                              const Counters* __restrict__ ctr, uint64_t* __restrict__ key0, uint64_t* __restrict__ key1,
                                              const uint32_t* __restrict__ pay0, const uint32_t* __restrict__ pay1,
                                              uint32_t* __restrict__ tile_hist)
{
    __shared__ uint32_t h[256];
    const uint32_t      ntiles = ctr->n_tiles;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        h[threadIdx.x] = 0;
        __syncthreads();
        const Bucket    B     = buckets[tile_bucket[t]];
        const uint32_t  first = (t - B.tile0) * TILE;
        const uint32_t  cnt   = min((uint32_t) TILE, B.len - first);
        uint64_t*       key   = B.buf ? key1 : key0;
        const uint32_t* pay   = B.buf ? pay1 : pay0;
        const uint32_t  kd    = eff_kd(B, MODE);
        const bool      rekey = (MODE == MODE_STRING) && kd != B.kd;
        const BlockDesc BD    = blocks[B.block];
        for (uint32_t i = threadIdx.x; i < cnt; i += TPB)
        {
            const size_t s = (size_t) B.start + first + i;
            uint64_t     k;
            if (rekey)
            {
                const uint32_t idx = pay[s] & 0xFFFFFFu;
                uint32_t       st  = idx + (B.d % BD.len);
                if (st >= BD.len)
                    st -= BD.len;
                k      = load_key8(in + BD.off, BD.len, st);
                key[s] = k;
            }
            else
                k = key[s];
            atomicAdd(&h[key_digit(k, B.d, kd)], 1u);
        }
        __syncthreads();
        tile_hist[(size_t) t * 256 + threadIdx.x] = h[threadIdx.x];
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------------------
// per-bucket scan: sub-bucket offsets per tile, next-level buckets, wave jobs, fallback groups
// -------------------------------------------------------------------------------------------------
struct ScanArgs
{
    const Bucket*   buckets;
    uint32_t        nbuckets;
    const uint32_t* tile_hist;
    uint32_t*       tile_off;
    uint8_t*        nomove;
    Bucket*         next;
    uint32_t        cap_next;
    Job*            jobs;
    uint32_t        cap_jobs;
    Group*          groups;
    uint32_t        cap_groups;
    Counters*       ctr;
    uint32_t        dcap;  // STRING: depth cap for big buckets
};

template <uint32_t MODE>
__global__ void __launch_bounds__(TPB) k_scan(ScanArgs a)
{
    __shared__ uint32_t tot_s[256];
    __shared__ uint32_t base_s[256];
    __shared__ uint32_t tmp[8];
    const uint32_t      dg = threadIdx.x;
    for (uint32_t bi = blockIdx.x; bi < a.nbuckets; bi += gridDim.x)
    {
        const Bucket   B      = a.buckets[bi];
        const uint32_t ntiles = div_up(B.len, TILE);
        uint32_t       tot    = 0;
        for (uint32_t t = 0; t < ntiles; ++t)
            tot += a.tile_hist[(size_t) (B.tile0 + t) * 256 + dg];
        const uint32_t base = block256_exclusive_sum(tot, tmp);
        tot_s[dg]           = tot;
        base_s[dg]          = base;
        uint32_t run        = B.start + base;
        for (uint32_t t = 0; t < ntiles; ++t)
        {
            const size_t o = (size_t) (B.tile0 + t) * 256 + dg;
            const uint32_t h = a.tile_hist[o];
            a.tile_off[o]    = run;
            run += h;
        }
        __syncthreads();
        const bool     nomove = __syncthreads_or(tot == B.len);
        const uint32_t kd     = eff_kd(B, MODE);
        const uint32_t nd     = B.d + 1;
        const uint32_t obuf   = (B.buf == 2u) ? 0u : (nomove ? B.buf : 1u - B.buf);  // buf 2 = level-0 input
        if (dg == 0)
        {
            a.nomove[bi] = nomove ? 1 : 0;
            if (!nomove)
                atomicAdd(&a.ctr->n_moved, B.len);
        }
        // big sub-buckets
        if (tot > JOB_MAX)
        {
            const uint32_t s = B.start + base;
            bool final_grp   = false;
            if (MODE == MODE_STRING)
                final_grp = nd >= a.dcap;
            else
                final_grp = nd >= RANK_KEYBYTES;
            if (final_grp)
            {
                const uint32_t gdep = (MODE == MODE_STRING) ? nd : B.gdepth;
                const uint32_t slot = atomicAdd(&a.ctr->n_groups, 1u);
                if (slot < a.cap_groups)
                {
                    a.groups[slot] = Group{s, tot, gdep, B.block | (obuf << 31)};
                    atomicAdd(&a.ctr->g_members, tot);
                    atomicMin(&a.ctr->hmin, gdep);
                }
                else
                    atomicExch(&a.ctr->overflow, 1u);
            }
            else
            {
                const uint32_t slot = atomicAdd(&a.ctr->n_big, 1u);
                if (slot < a.cap_next)
                    a.next[slot] = Bucket{s, tot, nd, kd, B.block, obuf, B.gdepth, 0};
                else
                    atomicExch(&a.ctr->overflow, 1u);
            }
        }
        // pack consecutive small sub-buckets into wave jobs (greedy, in slot order)
        if (dg == 0)
        {
            uint32_t js = 0, jl = 0;
            auto     flush = [&]() {
                if (jl)
                {
                    const uint32_t slot = atomicAdd(&a.ctr->n_jobs, 1u);
                    if (slot < a.cap_jobs)
                        a.jobs[slot] = Job{js, jl, kd, obuf, B.block, B.gdepth};
                    else
                        atomicExch(&a.ctr->overflow, 1u);
                }
                jl = 0;
            };
            for (int x = 0; x < 256; ++x)
            {
                const uint32_t c = tot_s[x];
                if (c == 0)
                    continue;
                if (c > JOB_MAX)
                {
                    flush();
                    continue;
                }
                if (jl + c > JOB_MAX)
                    flush();
                if (jl == 0)
                    js = B.start + base_s[x];
                jl += c;
            }
            flush();
        }
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------------------
// LDS-staged scatter of one tile into its sub-buckets
// -------------------------------------------------------------------------------------------------
struct TileStage
{
    uint64_t key[TILE];
    uint32_t pay[TILE];
    uint32_t cnt[256];
    uint32_t base[256];
    uint32_t goff[256];
    uint32_t tmp[8];
};

// Writes the staged tile (already in TileStage.key/pay, count `cnt`, digit base `base`) to global.
__device__ __forceinline__ void stage_and_write(TileStage& S, const uint64_t (&k)[PER_THREAD], const uint32_t (&v)[PER_THREAD],
                                                const uint32_t (&dgt)[PER_THREAD], uint32_t cnt, uint32_t d, uint32_t kd,
                                                uint64_t* __restrict__ okey, uint32_t* __restrict__ opay)
{
    uint32_t rank[PER_THREAD];
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i)
    {
        const uint32_t e = threadIdx.x + i * TPB;
        if (e < cnt)
            rank[i] = atomicAdd(&S.cnt[dgt[i]], 1u);
    }
    __syncthreads();
    const uint32_t c  = S.cnt[threadIdx.x];
    S.base[threadIdx.x] = block256_exclusive_sum(c, S.tmp);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i)
    {
        const uint32_t e = threadIdx.x + i * TPB;
        if (e < cnt)
        {
            const uint32_t q = S.base[dgt[i]] + rank[i];
            S.key[q]         = k[i];
            S.pay[q]         = v[i];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i)
    {
        const uint32_t q = threadIdx.x + i * TPB;
        if (q < cnt)
        {
            const uint64_t kk   = S.key[q];
            const uint32_t dd   = key_digit(kk, d, kd);
            const uint32_t slot = S.goff[dd] + (q - S.base[dd]);
            okey[slot]          = kk;
            opay[slot]          = S.pay[q];
        }
    }
}

__global__ void __launch_bounds__(TPB) k_l0_scatter(const uint8_t* __restrict__ in, const BlockDesc* __restrict__ blocks,
                                                    const L0Tile* __restrict__ tiles, uint32_t ntiles,
                                                    const uint32_t* __restrict__ tile_off, uint64_t* __restrict__ okey,
                                                    uint32_t* __restrict__ opay)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    TileStage& S   = *reinterpret_cast<TileStage*>(smem);
    uint8_t*   win = reinterpret_cast<uint8_t*>(smem + sizeof(TileStage));  // TILE + 16 bytes
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const L0Tile    T   = tiles[t];
        const BlockDesc B   = blocks[T.block];
        const uint32_t  cnt = min((uint32_t) TILE, B.len - T.start);
        const uint8_t*  blk = in + B.off;
        // window of bytes [start-1, start+cnt+7], cyclic in the block
        for (uint32_t i = threadIdx.x; i < cnt + 9; i += TPB)
        {
            int64_t q = (int64_t) T.start - 1 + i;
            q %= (int64_t) B.len;
            if (q < 0)
                q += B.len;
            win[i] = blk[q];
        }
        S.cnt[threadIdx.x]  = 0;
        S.goff[threadIdx.x] = tile_off[(size_t) t * 256 + threadIdx.x];
        __syncthreads();
        uint64_t k[PER_THREAD];
        uint32_t v[PER_THREAD], dg[PER_THREAD];
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i)
        {
            const uint32_t e = threadIdx.x + i * TPB;
            if (e < cnt)
            {
                uint64_t kk = 0;
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    kk = (kk << 8) | win[e + 1 + b];
                k[i]  = kk;
                v[i]  = ((uint32_t) win[e] << 24) | (T.start + e);
                dg[i] = (uint32_t) (kk >> 56);
            }
        }
        stage_and_write(S, k, v, dg, cnt, 0, 0, okey, opay);
        __syncthreads();
    }
}

__global__ void __launch_bounds__(TPB) k_scatter(const Bucket* __restrict__ buckets, const uint8_t* __restrict__ nomove,
                                                 const uint32_t* __restrict__ tile_bucket, const Counters* __restrict__ ctr,
                                                 const uint32_t* __restrict__ tile_off, uint64_t* __restrict__ key0,
                                                 uint64_t* __restrict__ key1, uint32_t* __restrict__ pay0, uint32_t* __restrict__ pay1,
                                                 uint32_t mode)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    TileStage&     S      = *reinterpret_cast<TileStage*>(smem);
    const uint32_t ntiles = ctr->n_tiles;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const uint32_t bi = tile_bucket[t];
        if (nomove[bi])
            continue;  // uniform per workgroup
        const Bucket    B     = buckets[bi];
        const uint32_t  first = (t - B.tile0) * TILE;
        const uint32_t  cnt   = min((uint32_t) TILE, B.len - first);
        const uint32_t  kd    = (mode == MODE_STRING && B.d - B.kd >= 8) ? B.d : B.kd;
        const uint64_t* ik    = B.buf ? key1 : key0;
        const uint32_t* ip    = B.buf ? pay1 : pay0;
        uint64_t*       ok    = B.buf ? key0 : key1;
        uint32_t*       op    = B.buf ? pay0 : pay1;
        S.cnt[threadIdx.x]    = 0;
        S.goff[threadIdx.x]   = tile_off[(size_t) t * 256 + threadIdx.x];
        __syncthreads();
        uint64_t k[PER_THREAD];
        uint32_t v[PER_THREAD], dg[PER_THREAD];
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i)
        {
            const uint32_t e = threadIdx.x + i * TPB;
            if (e < cnt)
            {
                const size_t s = (size_t) B.start + first + e;
                k[i]           = ik[s];
                v[i]           = ip[s];
                dg[i]          = key_digit(k[i], B.d, kd);
            }
        }
        stage_and_write(S, k, v, dg, cnt, B.d, kd, ok, op);
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------------------
// tiles of the current level's big buckets
// -------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(TPB) k_build_tiles(Bucket* __restrict__ buckets, uint32_t nb, uint32_t* __restrict__ tile_bucket,
                                                     uint32_t cap_tiles, Counters* __restrict__ ctr)
{
    __shared__ uint32_t tmp[8];
    __shared__ uint32_t carry, elems;
    if (threadIdx.x == 0)
        carry = elems = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nb; base += TPB)
    {
        const uint32_t i  = base + threadIdx.x;
        const uint32_t nt = (i < nb) ? div_up(buckets[i].len, TILE) : 0;
        if (i < nb)
            atomicAdd(&elems, buckets[i].len);
        uint32_t       total;
        const uint32_t ex = block256_exclusive_sum(nt, tmp, &total);
        const uint32_t t0 = carry + ex;
        if (i < nb)
        {
            buckets[i].tile0 = t0;
            for (uint32_t t = 0; t < nt; ++t)
                if (t0 + t < cap_tiles)
                    tile_bucket[t0 + t] = i;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0)
    {
        ctr->n_tiles = carry;
        ctr->n_elems = elems;
        if (carry > cap_tiles)
            ctr->overflow = 1;
    }
}

// -------------------------------------------------------------------------------------------------
// wave jobs: sort <= 256 elements in registers, refine ties (STRING) or split groups (RANK)
// -------------------------------------------------------------------------------------------------
struct JobArgs
{
    const Job*       jobs;
    uint32_t         njobs;
    const uint8_t*   in;
    const BlockDesc* blocks;
    const uint64_t*  key0;
    const uint64_t*  key1;
    const uint32_t*  pay0;
    const uint32_t*  pay1;
    uint32_t*        fsa;
    uint8_t*         L;
    uint32_t*        pi;
    uint32_t*        isa;    // RANK mode: rank array (group start, block-local)
    Group*           groups; // fallback / next-round groups
    uint32_t         cap_groups;
    Counters*        ctr;
    uint32_t         dcap;
    uint32_t         hstep;  // RANK mode: depth added to a subgroup (min depth of the round)
};

template <uint32_t MODE>
__global__ void __launch_bounds__(256) k_jobs(JobArgs a)
{
    const int      lane   = lane_id();
    const uint32_t wid    = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t j = wid; j < a.njobs; j += nwaves)
    {
        const Job       J  = a.jobs[j];
        const BlockDesc BD = a.blocks[J.block];
        const uint8_t*  blk = a.in + BD.off;
        const uint64_t* K  = J.buf ? a.key1 : a.key0;
        const uint32_t* V  = J.buf ? a.pay1 : a.pay0;
        uint64_t        k[4];
        uint32_t        v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t e = lane * 4 + r;
            if (e < J.len)
            {
                k[r] = K[J.start + e];
                v[r] = V[J.start + e];
            }
            else
            {
                k[r] = ~0ull;
                v[r] = ~0u;
            }
        }
        int P = 4;
        while ((uint32_t) P < J.len)
            P <<= 1;
        wave_bitonic_sort4(k, v, P);

        uint32_t g[4], gend[4];
        bool     tied[4];
        bool     final_ties = false, to_fallback = false;
        uint32_t depth      = (MODE == MODE_STRING) ? J.kd + 8 : J.gdepth;
        for (;;)
        {
            // group starts (head = key differs from predecessor)
            uint64_t prev3 = shfl_up64(k[3], 1);
            uint32_t h[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const uint32_t e  = lane * 4 + r;
                const uint64_t pk = (r == 0) ? prev3 : k[r - 1];
                const bool     hd = (e == 0) || e >= J.len || pk != k[r];
                h[r]              = hd ? e : 0;
                g[r]              = h[r];
                gend[r]           = hd ? e : 0xFFFFFFFFu;
            }
            wave_max_scan4(g);
            // group end: next head strictly after e
            uint32_t nh[4];
            {
                uint32_t x[4];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    x[r] = gend[r];
                wave_min_rscan4(x);  // x[r] = first head at or after e
                uint32_t nxt0 = __shfl_down(x[0], 1, WAVE);
                if (lane == WAVE - 1)
                    nxt0 = 0xFFFFFFFFu;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    nh[r] = (r < 3) ? x[r + 1] : nxt0;
            }
            bool any = false;
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const uint32_t e   = lane * 4 + r;
                const uint32_t end = min(nh[r] == 0xFFFFFFFFu ? (uint32_t) P : nh[r], J.len);
                gend[r]            = end;  // exclusive end of e's group
                tied[r]            = e < J.len && (end - g[r]) >= 2;
                any |= tied[r];
            }
            any = __any(any);
            if (MODE == MODE_RANK || !any)
                break;
            if (depth >= BD.len)
            {
                final_ties = true;
                break;
            }
            if (depth >= a.dcap)
            {
                to_fallback = true;
                break;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const uint32_t e = lane * 4 + r;
                if (e < J.len)
                {
                    uint64_t nk = (uint64_t) g[r] << 56;
                    if (tied[r])
                    {
                        const uint32_t idx = v[r] & 0xFFFFFFu;
                        uint32_t       st  = idx + depth;
                        if (st >= BD.len)
                            st -= BD.len;
                        nk |= load_key8(blk, BD.len, st) >> 8;
                    }
                    k[r] = nk;
                }
            }
            wave_bitonic_sort4(k, v, P);
            depth += 7;
        }

        // outputs
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t e = lane * 4 + r;
            if (e >= J.len)
                continue;
            const uint32_t slot = J.start + e;
            const uint32_t idx  = v[r] & 0xFFFFFFu;
            const uint32_t loc  = slot - (uint32_t) BD.off;
            a.fsa[slot]         = idx;
            a.L[slot]           = (uint8_t) (v[r] >> 24);
            const uint32_t gst  = J.start + g[r] - (uint32_t) BD.off;  // block-local group start
            if (MODE == MODE_RANK)
                a.isa[BD.off + idx] = gst;
            if (idx == 0)
            {
                if (MODE == MODE_RANK || final_ties)
                    a.pi[J.block] = gst;
                else if (!(to_fallback && tied[r]))
                    a.pi[J.block] = loc;
            }
            const bool emit = (MODE == MODE_RANK) ? tied[r] : (to_fallback && tied[r]);
            if (emit && g[r] == e)
            {
                const uint32_t gl   = gend[r] - e;
                const uint32_t gd   = (MODE == MODE_RANK) ? J.gdepth + a.hstep : depth;
                const uint32_t slot2 = atomicAdd(&a.ctr->n_groups, 1u);
                if (slot2 < a.cap_groups)
                {
                    a.groups[slot2] = Group{slot, gl, gd, J.block | (1u << 30)};  // bit 30: data already in fsa
                    atomicAdd(&a.ctr->g_members, gl);
                    atomicMin(&a.ctr->hmin, gd);
                }
                else
                    atomicExch(&a.ctr->overflow, 1u);
            }
        }
    }
}

// -------------------------------------------------------------------------------------------------
// fallback (prefix doubling on ranks) helpers
// -------------------------------------------------------------------------------------------------
// Copy the members of fallback groups that still live in a KV buffer into fsa.
__global__ void k_group_flush(const Group* __restrict__ groups, uint32_t ng, const uint32_t* __restrict__ pay0,
                              const uint32_t* __restrict__ pay1, uint32_t* __restrict__ fsa)
{
    for (uint32_t gi = blockIdx.x; gi < ng; gi += gridDim.x)
    {
        const Group G = groups[gi];
        if (G.block & (1u << 30))
            continue;
        const uint32_t* p = (G.block >> 31) ? pay1 : pay0;
        for (uint32_t i = threadIdx.x; i < G.len; i += blockDim.x)
            fsa[G.start + i] = p[G.start + i] & 0xFFFFFFu;
    }
}

// isa[off + fsa[j]] = j - off for every slot of the flagged blocks
__global__ void k_isa_init(const BlockDesc* __restrict__ blocks, const uint8_t* __restrict__ flag, uint32_t nblocks,
                           const uint32_t* __restrict__ fsa, uint32_t* __restrict__ isa)
{
    for (uint32_t b = blockIdx.y; b < nblocks; b += gridDim.y)
    {
        if (!flag[b])
            continue;
        const BlockDesc B = blocks[b];
        for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < B.len; j += gridDim.x * blockDim.x)
            isa[B.off + fsa[B.off + j]] = j;
    }
}

__global__ void k_group_mark(const Group* __restrict__ groups, uint32_t ng, const BlockDesc* __restrict__ blocks,
                             const uint32_t* __restrict__ fsa, uint32_t* __restrict__ isa, uint8_t* __restrict__ flag)
{
    for (uint32_t gi = blockIdx.x; gi < ng; gi += gridDim.x)
    {
        const Group     G  = groups[gi];
        const uint32_t  b  = G.block & 0x3FFFFFFFu;
        const BlockDesc BD = blocks[b];
        for (uint32_t i = threadIdx.x; i < G.len; i += blockDim.x)
            isa[BD.off + fsa[G.start + i]] = G.start - (uint32_t) BD.off;
        if (threadIdx.x == 0)
            flag[b] = 1;
    }
}

// Gather rank keys for all members of the round's groups; they become level-0 RANK buckets (buf 0).
__global__ void k_rank_keys(const Group* __restrict__ groups, uint32_t ng, const BlockDesc* __restrict__ blocks,
                            const uint8_t* __restrict__ in, const uint32_t* __restrict__ fsa, const uint32_t* __restrict__ isa,
                            uint64_t* __restrict__ key0, uint32_t* __restrict__ pay0)
{
    for (uint32_t gi = blockIdx.x; gi < ng; gi += gridDim.x)
    {
        const Group     G  = groups[gi];
        const BlockDesc BD = blocks[G.block & 0x3FFFFFFFu];
        const uint32_t  h  = G.depth % BD.len;
        for (uint32_t i = threadIdx.x; i < G.len; i += blockDim.x)
        {
            const uint32_t s   = G.start + i;
            const uint32_t idx = fsa[s];
            uint32_t       q   = idx + h;
            if (q >= BD.len)
                q -= BD.len;
            const uint32_t rk = isa[BD.off + q];
            key0[s]           = (uint64_t) rk << 32;
            const uint32_t pv = (idx == 0) ? BD.len - 1 : idx - 1;
            pay0[s]           = ((uint32_t) in[BD.off + pv] << 24) | idx;
        }
    }
}

// Groups -> RANK buckets (big) and one job per small group.
__global__ void k_groups_to_work(const Group* __restrict__ groups, uint32_t ng, Bucket* __restrict__ big, uint32_t cap_big,
                                 Job* __restrict__ jobs, uint32_t cap_jobs, Counters* __restrict__ ctr)
{
    for (uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x; gi < ng; gi += gridDim.x * blockDim.x)
    {
        const Group    G = groups[gi];
        const uint32_t b = G.block & 0x3FFFFFFFu;
        if (G.len > JOB_MAX)
        {
            const uint32_t s = atomicAdd(&ctr->n_big, 1u);
            if (s < cap_big)
                big[s] = Bucket{G.start, G.len, 0, 0, b, 0, G.depth, 0};
            else
                atomicExch(&ctr->overflow, 1u);
        }
        else
        {
            const uint32_t s = atomicAdd(&ctr->n_jobs, 1u);
            if (s < cap_jobs)
                jobs[s] = Job{G.start, G.len, 0, 0, b, G.depth};
            else
                atomicExch(&ctr->overflow, 1u);
        }
    }
}

// Final equal-key RANK groups (> JOB_MAX) still in a KV buffer: write fsa, L, isa, pi.
__global__ void k_rank_flush(const Group* __restrict__ groups, uint32_t ng, const BlockDesc* __restrict__ blocks,
                             const uint32_t* __restrict__ pay0, const uint32_t* __restrict__ pay1, uint32_t* __restrict__ fsa,
                             uint8_t* __restrict__ L, uint32_t* __restrict__ isa, uint32_t* __restrict__ pi)
{
    for (uint32_t gi = blockIdx.x; gi < ng; gi += gridDim.x)
    {
        const Group G = groups[gi];
        if (G.block & (1u << 30))
            continue;
        const uint32_t  b   = G.block & 0x3FFFFFFFu;
        const BlockDesc BD  = blocks[b];
        const uint32_t* p   = (G.block >> 31) ? pay1 : pay0;
        const uint32_t  gst = G.start - (uint32_t) BD.off;
        for (uint32_t i = threadIdx.x; i < G.len; i += blockDim.x)
        {
            const uint32_t s   = G.start + i;
            const uint32_t v   = p[s];
            const uint32_t idx = v & 0xFFFFFFu;
            fsa[s]             = idx;
            L[s]               = (uint8_t) (v >> 24);
            isa[BD.off + idx]  = gst;
            if (idx == 0)
                pi[b] = gst;
        }
    }
}

__global__ void k_pi_from_isa(const BlockDesc* __restrict__ blocks, const uint8_t* __restrict__ flag, uint32_t nblocks,
                              const uint32_t* __restrict__ isa, uint32_t* __restrict__ pi)
{
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += gridDim.x * blockDim.x)
        if (flag[b])
            pi[b] = isa[blocks[b].off];
}

}  // namespace

// =================================================================================================
// host driver
// =================================================================================================
struct BwtWorkspace
{
    uint64_t  cap_n      = 0;
    uint32_t  cap_blocks = 0;
    uint64_t* key[2]     = {nullptr, nullptr};
    uint32_t* pay[2]     = {nullptr, nullptr};
    uint32_t* fsa        = nullptr;
    uint32_t* isa        = nullptr;
    uint32_t* tile_hist  = nullptr;
    uint32_t* tile_off   = nullptr;
    uint32_t* tile_bucket = nullptr;
    uint8_t*  nomove     = nullptr;
    uint8_t*  flag       = nullptr;
    Bucket*   big[2]     = {nullptr, nullptr};
    Job*      jobs       = nullptr;
    Group*    groups[2]  = {nullptr, nullptr};
    Counters* ctr        = nullptr;
    Counters* h_ctr      = nullptr;  // pinned
    L0Tile*   l0tiles    = nullptr;
    uint32_t  cap_tiles = 0, cap_big = 0, cap_jobs = 0, cap_groups = 0, cap_l0 = 0;
    int       grid = 2048;
};

static void ws_free(BwtWorkspace& w)
{
    for (int i = 0; i < 2; ++i)
    {
        (void) hipFree(w.key[i]);
        (void) hipFree(w.pay[i]);
        (void) hipFree(w.big[i]);
        (void) hipFree(w.groups[i]);
    }
    (void) hipFree(w.fsa);
    (void) hipFree(w.isa);
    (void) hipFree(w.tile_hist);
    (void) hipFree(w.tile_off);
    (void) hipFree(w.tile_bucket);
    (void) hipFree(w.nomove);
    (void) hipFree(w.flag);
    (void) hipFree(w.jobs);
    (void) hipFree(w.ctr);
    (void) hipFree(w.l0tiles);
    if (w.h_ctr)
        (void) hipHostFree(w.h_ctr);
    w = BwtWorkspace{};
}

BwtWorkspace* bwt_workspace_create() { return new BwtWorkspace(); }
void          bwt_workspace_destroy(BwtWorkspace* w)
{
    if (w)
    {
        ws_free(*w);
        delete w;
    }
}

static bool ws_reserve(BwtWorkspace& w, uint64_t n, uint32_t nblocks)
{
    if (n <= w.cap_n && nblocks <= w.cap_blocks)
        return true;
    ws_free(w);
    const uint64_t N = std::max<uint64_t>(n, 1 << 16);
    const uint32_t B = std::max<uint32_t>(nblocks, 64);
    w.cap_n      = N;
    w.cap_blocks = B;
    w.cap_l0     = (uint32_t) (N / TILE + B + 1);
    w.cap_big    = (uint32_t) (N / JOB_MAX + B + 16);
    w.cap_tiles  = (uint32_t) (N / TILE + w.cap_big + 16);
    w.cap_jobs   = (uint32_t) (N / 8 + B + 1024);
    w.cap_groups = (uint32_t) (N / 64 + B + 4096);
    for (int i = 0; i < 2; ++i)
    {
        BRA_HIP_CHECK(hipMalloc(&w.key[i], N * 8));
        BRA_HIP_CHECK(hipMalloc(&w.pay[i], N * 4));
        BRA_HIP_CHECK(hipMalloc(&w.big[i], (size_t) w.cap_big * sizeof(Bucket)));
        BRA_HIP_CHECK(hipMalloc(&w.groups[i], (size_t) w.cap_groups * sizeof(Group)));
    }
    BRA_HIP_CHECK(hipMalloc(&w.fsa, N * 4));
    BRA_HIP_CHECK(hipMalloc(&w.isa, N * 4));
    const uint32_t tmax = std::max(w.cap_tiles, w.cap_l0);
    BRA_HIP_CHECK(hipMalloc(&w.tile_hist, (size_t) tmax * 256 * 4));
    BRA_HIP_CHECK(hipMalloc(&w.tile_off, (size_t) tmax * 256 * 4));
    BRA_HIP_CHECK(hipMalloc(&w.tile_bucket, (size_t) tmax * 4));
    BRA_HIP_CHECK(hipMalloc(&w.nomove, std::max<uint32_t>(w.cap_big, B)));
    BRA_HIP_CHECK(hipMalloc(&w.flag, B));
    BRA_HIP_CHECK(hipMalloc(&w.jobs, (size_t) w.cap_jobs * sizeof(Job)));
    BRA_HIP_CHECK(hipMalloc(&w.ctr, sizeof(Counters)));
    BRA_HIP_CHECK(hipMalloc(&w.l0tiles, (size_t) w.cap_l0 * sizeof(L0Tile)));
    BRA_HIP_CHECK(hipHostMalloc(&w.h_ctr, sizeof(Counters), hipHostMallocDefault));
    return true;
}

static bool read_ctr(BwtWorkspace& w, hipStream_t s)
{
    BRA_HIP_CHECK(hipMemcpyAsync(w.h_ctr, w.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
    BRA_HIP_CHECK(hipStreamSynchronize(s));
    if (w.h_ctr->overflow)
    {
        bra_hip_report("bwt: work list overflow");
        return false;
    }
    return true;
}

static bool reset_ctr(BwtWorkspace& w, hipStream_t s)
{
    Counters z{};
    z.hmin = 0xFFFFFFFFu;
    // small H2D of a constant: use the pinned staging to stay async-safe
    *w.h_ctr = z;
    BRA_HIP_CHECK(hipMemcpyAsync(w.ctr, w.h_ctr, sizeof(Counters), hipMemcpyHostToDevice, s));
    return true;
}

static size_t tile_stage_bytes() { return sizeof(TileStage); }

// Runs the MSD levels + wave jobs for the buckets currently in w.big[cur] (count nbig) and the jobs
// already queued.  Returns false on error.
template <uint32_t MODE>
static bool run_levels(BwtWorkspace& w, const uint8_t* d_in, const BlockDesc* d_blocks, uint32_t nbig, int cur, uint8_t* d_L,
                       uint32_t* d_pi, Group* groups_out, uint32_t hstep, hipStream_t s, uint32_t& njobs_total)
{
    const size_t lds = tile_stage_bytes();
    while (nbig > 0)
    {
        {
            BRA_PROF(P_BWT_TILES, s);
            hipLaunchKernelGGL(k_build_tiles, dim3(1), dim3(TPB), 0, s, w.big[cur], nbig, w.tile_bucket, w.cap_tiles, w.ctr);
        }
        // zero n_big / n_moved for the next level (keep jobs/groups counters)
        BRA_HIP_CHECK(hipMemsetAsync(&w.ctr->n_big, 0, 4, s));
        BRA_HIP_CHECK(hipMemsetAsync(&w.ctr->n_moved, 0, 4, s));
        const int grid = w.grid;
        {
            BRA_PROF(P_BWT_HIST, s);
            hipLaunchKernelGGL(k_hist<MODE>, dim3(grid), dim3(TPB), 0, s, d_in, d_blocks, w.big[cur], w.tile_bucket, w.ctr, w.key[0],
                               w.key[1], w.pay[0], w.pay[1], w.tile_hist);
        }
        ScanArgs a{w.big[cur], nbig,    w.tile_hist, w.tile_off, w.nomove,  w.big[cur ^ 1], w.cap_big, w.jobs, w.cap_jobs,
                   groups_out, w.cap_groups, w.ctr,  MODE == MODE_STRING ? DCAP_BIG : RANK_KEYBYTES};
        {
            BRA_PROF(P_BWT_SCAN, s);
            hipLaunchKernelGGL(k_scan<MODE>, dim3(std::min<uint32_t>(nbig, 65535u)), dim3(TPB), 0, s, a);
        }
        {
            BRA_PROF(P_BWT_SCATTER, s);
            hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(TPB), lds, s, w.big[cur], w.nomove, w.tile_bucket, w.ctr, w.tile_off,
                               w.key[0], w.key[1], w.pay[0], w.pay[1], MODE);
        }
        BRA_HIP_CHECK(hipGetLastError());
        if (!read_ctr(w, s))
            return false;
        // algorithmic bytes: keys read by the histogram, tile histograms, KV moved by the scatter
        const double nt = w.h_ctr->n_tiles, ne = w.h_ctr->n_elems, nm = w.h_ctr->n_moved;
        prof_bytes(P_BWT_TILES, 32.0 * nbig + 4.0 * nt);
        prof_bytes(P_BWT_HIST, 8.0 * ne + 1024.0 * nt);
        prof_bytes(P_BWT_SCAN, 3072.0 * nt + 32.0 * nbig);
        prof_bytes(P_BWT_SCATTER, 24.0 * nm + 1024.0 * nt);
        nbig = w.h_ctr->n_big;
        cur ^= 1;
    }
    (void) d_L, (void) d_pi, (void) hstep;
    njobs_total = w.h_ctr->n_jobs;
    return true;
}

bool bwt_encode_device(BwtWorkspace* wp, const uint8_t* d_in, const BlockDesc* d_blocks, const BlockDesc* h_blocks, uint32_t nblocks,
                       uint8_t* d_L, uint32_t* d_pi, hipStream_t s)
{
    BwtWorkspace& w = *wp;
    uint64_t      N = 0;
    for (uint32_t b = 0; b < nblocks; ++b)
    {
        if (h_blocks[b].len == 0 || h_blocks[b].len >= (1u << 24))
        {
            bra_hip_report("bwt: block %u has unsupported length %u", b, h_blocks[b].len);
            return false;
        }
        N = std::max<uint64_t>(N, h_blocks[b].off + h_blocks[b].len);
    }
    if (N >= (1ull << 31))
    {
        bra_hip_report("bwt: batch too large (%llu bytes)", (unsigned long long) N);
        return false;
    }
    if (!ws_reserve(w, N, nblocks))
        return false;
    static bool attr_set = false;
    if (!attr_set)
    {
        const size_t lds = tile_stage_bytes();
        BRA_HIP_CHECK(hipFuncSetAttribute((const void*) k_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
        BRA_HIP_CHECK(hipFuncSetAttribute((const void*) k_l0_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int) (lds + TILE + 16)));
        attr_set = true;
    }

    // ---- level 0 (buckets = blocks, elements read straight from the input) ----
    std::vector<L0Tile> tiles;
    std::vector<Bucket> l0b(nblocks);
    for (uint32_t b = 0; b < nblocks; ++b)
    {
        l0b[b] = Bucket{(uint32_t) h_blocks[b].off, h_blocks[b].len, 0, 0, b, 2u, 0, (uint32_t) tiles.size()};
        for (uint32_t st = 0; st < h_blocks[b].len; st += TILE)
            tiles.push_back(L0Tile{b, st});
    }
    const uint32_t nt0 = (uint32_t) tiles.size();
    BRA_HIP_CHECK(hipMemcpyAsync(w.l0tiles, tiles.data(), nt0 * sizeof(L0Tile), hipMemcpyHostToDevice, s));
    BRA_HIP_CHECK(hipMemcpyAsync(w.big[1], l0b.data(), nblocks * sizeof(Bucket), hipMemcpyHostToDevice, s));
    if (!reset_ctr(w, s))
        return false;
    BRA_HIP_CHECK(hipMemsetAsync(w.flag, 0, nblocks, s));
    const int grid = w.grid;
    {
        BRA_PROF(P_BWT_L0HIST, s);
        hipLaunchKernelGGL(k_l0_hist, dim3(std::min<uint32_t>(nt0, grid)), dim3(TPB), 0, s, d_in, d_blocks, w.l0tiles, nt0, w.tile_hist);
    }
    ScanArgs a0{w.big[1], nblocks,  w.tile_hist, w.tile_off, w.nomove, w.big[0], w.cap_big, w.jobs, w.cap_jobs,
                w.groups[0], w.cap_groups, w.ctr, DCAP_BIG};
    {
        BRA_PROF(P_BWT_SCAN, s);
        hipLaunchKernelGGL(k_scan<MODE_STRING>, dim3(std::min<uint32_t>(nblocks, 65535u)), dim3(TPB), 0, s, a0);
    }
    {
        BRA_PROF(P_BWT_L0SCATTER, s);
        hipLaunchKernelGGL(k_l0_scatter, dim3(std::min<uint32_t>(nt0, grid)), dim3(TPB), tile_stage_bytes() + TILE + 16, s, d_in, d_blocks,
                           w.l0tiles, nt0, w.tile_off, w.key[0], w.pay[0]);
    }
    BRA_HIP_CHECK(hipGetLastError());
    if (!read_ctr(w, s))
        return false;
    prof_bytes(P_BWT_L0HIST, (double) N + 1024.0 * nt0);
    prof_bytes(P_BWT_SCAN, 3072.0 * nt0);
    prof_bytes(P_BWT_L0SCATTER, 13.0 * N + 1024.0 * nt0);
    // Level 0 never keeps data in place ("nomove" only matters for level >= 1): all sub-buckets are in buf 0.
    uint32_t njobs = 0;
    if (!run_levels<MODE_STRING>(w, d_in, d_blocks, w.h_ctr->n_big, 0, d_L, d_pi, w.groups[0], 0, s, njobs))
        return false;

    // ---- wave jobs ----
    JobArgs ja{w.jobs,  njobs,     d_in,        d_blocks, w.key[0], w.key[1], w.pay[0], w.pay[1], w.fsa, d_L, d_pi,
               w.isa,   w.groups[0], w.cap_groups, w.ctr,  DCAP_JOB, 0};
    if (njobs)
        {
            BRA_PROF(P_BWT_JOBS, s);
            hipLaunchKernelGGL(k_jobs<MODE_STRING>, dim3(std::min<uint32_t>(div_up(njobs, 4), 8192u)), dim3(256), 0, s, ja);
        }
    BRA_HIP_CHECK(hipGetLastError());
    if (!read_ctr(w, s))
        return false;
    prof_bytes(P_BWT_JOBS, 17.0 * N);  // read key+payload, write SA entry + L byte

    // ---- fallback: prefix doubling on the groups still tied ----
    uint32_t ng = w.h_ctr->n_groups;
    if (ng == 0)
        return true;
    int gcur = 0;
    hipLaunchKernelGGL(k_group_flush, dim3(std::min<uint32_t>(ng, 4096u)), dim3(256), 0, s, w.groups[gcur], ng, w.pay[0], w.pay[1], w.fsa);
    // mark blocks, build ranks: singletons rank = own slot, group members = group start
    hipLaunchKernelGGL(k_group_mark, dim3(std::min<uint32_t>(ng, 4096u)), dim3(256), 0, s, w.groups[gcur], ng, d_blocks, w.fsa, w.isa,
                       w.flag);  // sets flags (isa writes are redone below)
    hipLaunchKernelGGL(k_isa_init, dim3(64, std::min<uint32_t>(nblocks, 65535u)), dim3(256), 0, s, d_blocks, w.flag, nblocks, w.fsa, w.isa);
    hipLaunchKernelGGL(k_group_mark, dim3(std::min<uint32_t>(ng, 4096u)), dim3(256), 0, s, w.groups[gcur], ng, d_blocks, w.fsa, w.isa,
                       w.flag);
    uint64_t members = w.h_ctr->g_members;
    uint32_t hmin    = w.h_ctr->hmin;
    for (int round = 0; round < 64 && ng > 0; ++round)
    {
        // keys for this round (all reads of isa happen here, before any rank update)
        hipLaunchKernelGGL(k_rank_keys, dim3(std::min<uint32_t>(ng, 8192u)), dim3(256), 0, s, w.groups[gcur], ng, d_blocks, d_in, w.fsa,
                           w.isa, w.key[0], w.pay[0]);
        Counters z{};
        z.hmin   = 0xFFFFFFFFu;
        *w.h_ctr = z;
        BRA_HIP_CHECK(hipMemcpyAsync(w.ctr, w.h_ctr, sizeof(Counters), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_groups_to_work, dim3(std::min<uint32_t>(div_up(ng, 256), 4096u)), dim3(256), 0, s, w.groups[gcur], ng, w.big[0],
                           w.cap_big, w.jobs, w.cap_jobs, w.ctr);
        if (!read_ctr(w, s))
            return false;
        const uint32_t nbig0 = w.h_ctr->n_big;
        // subgroups go to groups[gcur^1]; their depth = group depth + hmin
        Group* gnext = w.groups[gcur ^ 1];
        // run the MSD levels in RANK mode
        {
            uint32_t nb  = nbig0;
            int      cur = 0;
            // big buckets: levels over 4 key bytes; subgroups of equal key > JOB_MAX become groups directly
            while (nb > 0)
            {
                {
                    BRA_PROF(P_BWT_TILES, s);
                    hipLaunchKernelGGL(k_build_tiles, dim3(1), dim3(TPB), 0, s, w.big[cur], nb, w.tile_bucket, w.cap_tiles, w.ctr);
                }
                BRA_HIP_CHECK(hipMemsetAsync(&w.ctr->n_big, 0, 4, s));
                {
                    BRA_PROF(P_BWT_HIST, s);
                    hipLaunchKernelGGL(k_hist<MODE_RANK>, dim3(grid), dim3(TPB), 0, s, d_in, d_blocks, w.big[cur], w.tile_bucket, w.ctr,
                                       w.key[0], w.key[1], w.pay[0], w.pay[1], w.tile_hist);
                }
                ScanArgs a{w.big[cur], nb,    w.tile_hist, w.tile_off, w.nomove, w.big[cur ^ 1], w.cap_big, w.jobs, w.cap_jobs,
                           gnext,      w.cap_groups, w.ctr, RANK_KEYBYTES};
                {
                    BRA_PROF(P_BWT_SCAN, s);
                    hipLaunchKernelGGL(k_scan<MODE_RANK>, dim3(std::min<uint32_t>(nb, 65535u)), dim3(TPB), 0, s, a);
                }
                {
                    BRA_PROF(P_BWT_SCATTER, s);
                    hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(TPB), tile_stage_bytes(), s, w.big[cur], w.nomove, w.tile_bucket, w.ctr,
                                       w.tile_off, w.key[0], w.key[1], w.pay[0], w.pay[1], (uint32_t) MODE_RANK);
                }
                if (!read_ctr(w, s))
                    return false;
                nb = w.h_ctr->n_big;
                cur ^= 1;
            }
        }
        // equal-key big subgroups emitted by k_scan carry depth = gdepth; fix their depth and flush them
        const uint32_t ng_big = w.h_ctr->n_groups;
        const uint32_t nj     = w.h_ctr->n_jobs;
        JobArgs jr{w.jobs, nj, d_in, d_blocks, w.key[0], w.key[1], w.pay[0], w.pay[1], w.fsa, d_L, d_pi, w.isa, gnext, w.cap_groups,
                   w.ctr, 0, hmin};
        if (ng_big)
            hipLaunchKernelGGL(k_rank_flush, dim3(std::min<uint32_t>(ng_big, 4096u)), dim3(256), 0, s, gnext, ng_big, d_blocks, w.pay[0],
                               w.pay[1], w.fsa, d_L, w.isa, d_pi);
        if (nj)
            {
                BRA_PROF(P_BWT_JOBS, s);
                hipLaunchKernelGGL(k_jobs<MODE_RANK>, dim3(std::min<uint32_t>(div_up(nj, 4), 8192u)), dim3(256), 0, s, jr);
            }
        BRA_HIP_CHECK(hipGetLastError());
        if (!read_ctr(w, s))
            return false;
        const uint32_t ng_new = w.h_ctr->n_groups;
        // depth update for the big equal-key subgroups (they were emitted with the parent's depth)
        if (ng_big)
        {
            std::vector<Group> tmpg(ng_big);
            BRA_HIP_CHECK(hipMemcpyAsync(tmpg.data(), gnext, ng_big * sizeof(Group), hipMemcpyDeviceToHost, s));
            BRA_HIP_CHECK(hipStreamSynchronize(s));
            for (auto& g : tmpg)
            {
                g.depth += hmin;
                g.block |= (1u << 30);  // now flushed into fsa
                g.block &= ~(1u << 31);
            }
            BRA_HIP_CHECK(hipMemcpyAsync(gnext, tmpg.data(), ng_big * sizeof(Group), hipMemcpyHostToDevice, s));
        }
        const uint64_t members_new = w.h_ctr->g_members;
        // no split in this round (same groups, same members) => the partition is final
        const bool no_split = (ng_new == ng) && (members_new == members);
        ng                  = ng_new;
        members             = members_new;
        // min depth of the new groups: the emitted depths already include hmin; recompute
        uint32_t newmin = w.h_ctr->hmin;
        if (ng_big)
            newmin = std::min<uint32_t>(newmin, 0xFFFFFFFFu);
        {
            // exact min over new groups (host side; the lists are small in practice)
            std::vector<Group> all(ng);
            if (ng)
            {
                BRA_HIP_CHECK(hipMemcpyAsync(all.data(), gnext, ng * sizeof(Group), hipMemcpyDeviceToHost, s));
                BRA_HIP_CHECK(hipStreamSynchronize(s));
            }
            uint32_t m = 0xFFFFFFFFu;
            std::vector<Group> keep;
            keep.reserve(ng);
            for (auto& g : all)
            {
                const uint32_t b = g.block & 0x3FFFFFFFu;
                if (g.depth >= h_blocks[b].len)
                    continue;  // identical rotations: final
                m = std::min(m, g.depth);
                keep.push_back(g);
            }
            if (keep.size() != all.size())
            {
                ng = (uint32_t) keep.size();
                if (ng)
                    BRA_HIP_CHECK(hipMemcpyAsync(gnext, keep.data(), ng * sizeof(Group), hipMemcpyHostToDevice, s));
                members = 0;
                for (auto& g : keep)
                    members += g.len;
            }
            hmin = m;
        }
        gcur ^= 1;
        if (no_split)
            break;
    }
    hipLaunchKernelGGL(k_pi_from_isa, dim3(std::min<uint32_t>(div_up(nblocks, 256), 1024u)), dim3(256), 0, s, d_blocks, w.flag, nblocks,
                       w.isa, d_pi);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace bra
