// ibwt.hip -- inverse BWT for a batch of independent blocks.
//
// Replaces bra_bwt_decode2 (reference src/encoders/bra_bwt.c:133-168): transform[first[c]+k] = the
// position of the k-th c in L (a stable partition of positions by byte, :141-159), then n steps
// `index = transform[index]; out[i] = L[index]` starting at the primary index (:161-167).
//
// The pointer chase is split with splitters: every SPL-th transform index plus the primary index.
// Each splitter's thread walks to the next splitter (pass 1, recording the hop and its length),
// one lane per block chains the hops from the primary index in LDS to get output offsets, and the
// walkers re-walk writing their output (pass 3).  A primary index on a cycle shorter than n (a
// periodic block) makes the output periodic with that cycle length, exactly like the reference.
#include "ibwt.h"

namespace bra {

namespace {

constexpr int      TPB        = 256;
constexpr uint32_t MAX_SPLIT  = 4096;  // splitters per block (+1 for the primary index)
constexpr uint32_t ITILE      = 4096;

__device__ __forceinline__ uint32_t split_step(uint32_t n)
{
    uint32_t s = 256;
    while ((n + s - 1) / s > MAX_SPLIT)
        s <<= 1;
    return s;
}

// per tile byte histogram of L
__global__ void __launch_bounds__(TPB) k_ib_hist(const uint8_t* __restrict__ L, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                 uint32_t* __restrict__ th)
{
    __shared__ uint32_t h[256];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        h[threadIdx.x] = 0;
        __syncthreads();
        const Piece P = tiles[t];
        for (uint32_t i = threadIdx.x; i < P.len; i += TPB)
            atomicAdd(&h[L[P.off + i]], 1u);
        __syncthreads();
        th[(size_t) t * 256 + threadIdx.x] = h[threadIdx.x];
        __syncthreads();
    }
}

// per block: tile offsets per byte = first[c] + sum over earlier tiles
__global__ void __launch_bounds__(TPB) k_ib_scan(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count, uint32_t nblocks,
                                                 uint32_t* __restrict__ th)
{
    __shared__ uint32_t tmp[8];
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t t0 = first[b], nt = count[b], c = threadIdx.x;
        uint32_t       tot = 0;
        for (uint32_t i = 0; i < nt; ++i)
            tot += th[(size_t) (t0 + i) * 256 + c];
        uint32_t run = block256_exclusive_sum(tot, tmp);
        for (uint32_t i = 0; i < nt; ++i)
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
    const int           lane = lane_id();
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const Piece P = tiles[t];
        for (int i = lane; i < 256; i += 64)
            cnt[i] = th[(size_t) t * 256 + i];
        __syncthreads();
        const uint64_t boff = blocks[P.block].off;
        for (uint32_t base = 0; base < P.len; base += 64)
        {
            const uint32_t i     = base + lane;
            const bool     valid = i < P.len;
            const uint32_t c     = valid ? L[P.off + i] : 0xFFFFFFFFu;
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
        if (!dev_alloc(th, (uint64_t) c * 256))
            return false;
        cap_t = c;
    }
    if (nblocks > cap_b)
    {
        cap_b            = 0;
        const uint32_t c = nblocks + 8;
        if (!dev_alloc(hop_next, (uint64_t) c * (MAX_SPLIT + 1)) || !dev_alloc(hop_len, (uint64_t) c * (MAX_SPLIT + 1)) ||
            !dev_alloc(start, (uint64_t) c * (MAX_SPLIT + 1)) || !dev_alloc(cyc, c))
            return false;
        cap_b = c;
    }
    return true;
}

void IbwtWorkspace::release()
{
    tiling.release();
    (void) hipFree(T);
    (void) hipFree(th);
    (void) hipFree(hop_next);
    (void) hipFree(hop_len);
    (void) hipFree(start);
    (void) hipFree(cyc);
    *this = IbwtWorkspace{};
}

bool ibwt_device(IbwtWorkspace& w, const uint8_t* d_L, const uint32_t* d_pi, const BlockDesc* d_blocks, const BlockDesc* h_blocks,
                 uint32_t nblocks, uint8_t* d_out, hipStream_t s)
{
    if (!w.tiling.build(h_blocks, nblocks, ITILE, s))
        return false;
    uint64_t N = 0;
    for (uint32_t b = 0; b < nblocks; ++b)
        N = std::max<uint64_t>(N, h_blocks[b].off + h_blocks[b].len);
    const uint32_t nt = w.tiling.n;
    if (!w.reserve(N, nblocks, nt))
        return false;
    hipLaunchKernelGGL(k_ib_hist, dim3(std::min<uint32_t>(nt, 8192)), dim3(TPB), 0, s, d_L, w.tiling.d_pieces, nt, w.th);
    hipLaunchKernelGGL(k_ib_scan, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(TPB), 0, s, w.tiling.d_first, w.tiling.d_count, nblocks, w.th);
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

}  // namespace bra
