// huffman.hip -- canonical Huffman coding for a batch of independent blocks.
//
// Replaces bra_huffman_encode / bra_huffman_decode (reference src/encoders/bra_huffman.c:352-432,
// :434-498).  Encode:
//   k_huff_build     one wave per block: code lengths from the reference's frequency-sorted list
//                    (bra_minHeap_insert :90-118 restated as: position 0 if the head's frequency is
//                    larger, else max(1, lower_bound(f)); leaves inserted in symbol order :140-153;
//                    merge = pop l, pop r, insert l+r :158-175) kept in registers, leaf depth by
//                    pointer jumping, canonical codes in uint32 with wrap (:227-261, closed form +
//                    per-length ranks), bit count and encoded size (:389-395).  Single-leaf trees
//                    get length 1 (:201-207).
//   k_huff_offsets   exclusive scan of the encoded sizes -> byte offset of each block's payload
//   k_huff_tilebits  bits of each 4096-symbol tile of a block's RLE output
//   k_huff_tilescan  per block: bit offset of every tile
//   k_huff_zero      zero the words at tile boundaries (they are OR-ed by two tiles)
//   k_huff_pack      codes written MSB-first (:405-428) into an LDS word image of the tile, stored
//                    with plain stores inside the tile and atomicOr on the two boundary words.
// Decode: per block the reference's decode tree (:263-348: canonical codes inserted bit by bit,
// a leaf that gains children stops being a leaf) is rebuilt on the device, turned into an 11-bit
// primary lookup table, and walked (:455-482) with the reference's stop rule and error cases.
#include "huffman.h"
#include "prof.h"

namespace bra {

namespace {

constexpr int TPB = 256;

// ------------------------------------------------------------------------------------------------
// code lengths + canonical codes (one wave per block)
// ------------------------------------------------------------------------------------------------
// Whole-wave lane shifts (DPP wave_shr:1 / wave_shl:1): lane i gets lane i - 1 / i + 1; the lane
// without a source keeps 0.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) { return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x138, 0xF, 0xF, false); }
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v) { return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x130, 0xF, 0xF, false); }

struct BuildLds
{
    uint32_t node_f[512];
    uint16_t parent[512];
    uint32_t cnt[260];
    uint32_t next[260];
    uint8_t  len_s[256];
};

__global__ void __launch_bounds__(64) k_huff_build(const uint32_t* __restrict__ hist, const uint32_t* __restrict__ rle_size,
                                                   uint32_t nblocks, HuffMetaRec* __restrict__ meta, uint32_t* __restrict__ codes)
{
    __shared__ BuildLds S;
    const int           lane = lane_id();
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t* H = hist + (size_t) b * 256;
        uint32_t        h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            h[r] = H[lane * 4 + r];
        // leaves: ids in symbol order
        uint32_t nz = (h[0] != 0) + (h[1] != 0) + (h[2] != 0) + (h[3] != 0);
        uint32_t ex = nz;
        for (int d = 1; d < 64; d <<= 1)
        {
            uint32_t o = __shfl_up(ex, d, 64);
            if (lane >= d)
                ex += o;
        }
        const uint32_t leaves = __shfl(ex, 63, 64);
        ex -= nz;
        {
            uint32_t id = ex;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (h[r])
                {
                    S.node_f[id] = h[r];
                    S.parent[id] = 0xFFFF;
                    ++id;
                }
        }
        __syncthreads();
        // The frequency-sorted list lives in registers: position j = 64 r + lane (at most 256
        // entries).  An insert or a merge is ballots + lane shuffles -- no LDS round trips or
        // barriers per step (the LDS list cost 0.35 ms per 256-block batch, one wave per block
        // on an otherwise idle GPU).
        uint32_t LF[4] = {0, 0, 0, 0}, LI[4] = {0, 0, 0, 0}, len = 0;
        const auto lt_count = [&](uint32_t f, uint32_t from) {  // entries in [from, len) with frequency < f
            uint32_t c = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                if (64u * r >= len)
                    break;
                const uint32_t j = 64u * r + lane;
                c += (uint32_t) __builtin_popcountll(__builtin_amdgcn_ballot_w64(j >= from && j < len && LF[r] < f));
            }
            return c;
        };
        // Leaves in symbol order (:140-153): position 0 if the head's frequency is larger, else
        // max(1, entries with a smaller frequency) (:90-118).  The list stays sorted by frequency,
        // so the insertions have a closed form, computed for all leaves at once instead of one
        // insertion (ballots + lane shifts) per leaf: a leaf's position = the leaves of smaller
        // frequency + its rank among its equals.  Equals go in front of each other (lower bound),
        // except while their frequency is the smallest seen so far (no earlier symbol is rarer):
        // those land at position 1, right behind the group's first leaf.  With the group's members
        // x1..xm in symbol order and x1..xk inserted in that regime the group reads
        // xm .. x(k+1), x1, xk .. x2 (k = 0: xm .. x1).
        {
            uint32_t less[4] = {0, 0, 0, 0}, eq[4] = {0, 0, 0, 0}, eqb[4] = {0, 0, 0, 0}, lessb[4] = {0, 0, 0, 0}, lid[4];
            {
                uint32_t id = ex;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    lid[r] = h[r] ? id++ : 0xFFFFFFFFu;
            }
            for (uint32_t q = 0; q < leaves; ++q)
            {
                const uint32_t fq = S.node_f[q];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                {
                    less[r] += fq < h[r] ? 1u : 0u;
                    eq[r] += fq == h[r] ? 1u : 0u;
                    eqb[r] += (fq == h[r] && q < lid[r]) ? 1u : 0u;
                    lessb[r] += (fq < h[r] && q < lid[r]) ? 1u : 0u;
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (h[r])
                    S.next[lid[r]] = lessb[r] == 0 ? 1u : 0u;  // inserted while the smallest so far
            __syncthreads();
            uint32_t kmin[4] = {0, 0, 0, 0};
            for (uint32_t q = 0; q < leaves; ++q)
            {
                const uint32_t fq = S.node_f[q], mq = S.next[q];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    kmin[r] += (fq == h[r] && mq) ? 1u : 0u;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (h[r])
                {
                    const uint32_t m = eq[r], i = eqb[r] + 1, k = kmin[r];
                    const uint32_t rank = k == 0 ? m - i : (i == 1 ? m - k : (i <= k ? m - i + 1 : m - i));
                    S.cnt[less[r] + rank]   = h[r];            // (cnt / len_s: free until the lengths)
                    S.len_s[less[r] + rank] = (uint8_t) lid[r];
                }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const uint32_t j = 64u * r + lane;
                LF[r]            = j < leaves ? S.cnt[j] : 0u;
                LI[r]            = j < leaves ? (uint32_t) S.len_s[j] : 0u;
            }
            len = leaves;
            __syncthreads();
        }
        // merges (:158-175): pop the two head entries, insert their sum by the same rule
        uint32_t nodes = leaves;
        while (len > 1)
        {
            const uint32_t f  = __builtin_amdgcn_readlane(LF[0], 0) + __builtin_amdgcn_readlane(LF[0], 1);
            const uint32_t l  = __builtin_amdgcn_readlane(LI[0], 0), rt = __builtin_amdgcn_readlane(LI[0], 1);
            const uint32_t id = nodes++;
            if (lane == 0)
            {
                S.parent[id] = 0xFFFF;
                S.parent[l]  = (uint16_t) id;
                S.parent[rt] = (uint16_t) id;
            }
            // the list after the pops is old positions [2, len); new[j] = old[j + 2] below the
            // insert position p, the new node at p, old[j + 1] above
            const uint32_t n2    = len - 2;
            const uint32_t headf = __builtin_amdgcn_readlane(LF[0], 2);
            const uint32_t lt    = lt_count(f, 2);
            const uint32_t p     = (n2 == 0 || headf > f) ? 0u : (lt > 1u ? lt : 1u);
            uint32_t       d2F[4], d1F[4], d2I[4], d1I[4], n0F[4], n1F[4], n0I[4], n1I[4];
            const int      nr = (int) ((len - 1) / 64u) + 1;  // registers holding the list before the pops
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                if (r >= nr)
                    break;
                d1F[r] = wave_shl1(LF[r]);
                d2F[r] = wave_shl1(d1F[r]);
                d1I[r] = wave_shl1(LI[r]);
                d2I[r] = wave_shl1(d1I[r]);
                const int q = r < 3 ? r + 1 : 3;
                n0F[r] = r < 3 ? (uint32_t) __builtin_amdgcn_readlane(LF[q], 0) : 0u;
                n1F[r] = r < 3 ? (uint32_t) __builtin_amdgcn_readlane(LF[q], 1) : 0u;
                n0I[r] = r < 3 ? (uint32_t) __builtin_amdgcn_readlane(LI[q], 0) : 0u;
                n1I[r] = r < 3 ? (uint32_t) __builtin_amdgcn_readlane(LI[q], 1) : 0u;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                if (r >= nr)
                    break;
                const uint32_t j  = 64u * r + lane;
                const uint32_t aF = lane < 62 ? d2F[r] : (lane == 62 ? n0F[r] : n1F[r]);
                const uint32_t aI = lane < 62 ? d2I[r] : (lane == 62 ? n0I[r] : n1I[r]);
                const uint32_t bF = lane < 63 ? d1F[r] : n0F[r];
                const uint32_t bI = lane < 63 ? d1I[r] : n0I[r];
                LF[r]             = j < p ? aF : (j == p ? f : bF);
                LI[r]             = j < p ? aI : (j == p ? id : bI);
            }
            len = n2 + 1;
        }
        __syncthreads();
        // depth of every node by pointer jumping (root has parent 0xFFFF, depth 0)
        uint32_t anc[8], dep[8];
#pragma unroll
        for (int r = 0; r < 8; ++r)
        {
            const uint32_t v = lane + 64 * r;
            if (v < nodes)
            {
                anc[r] = S.parent[v];
                dep[r] = anc[r] == 0xFFFF ? 0 : 1;
            }
        }
        __syncthreads();
        for (int it = 0; it < 9; ++it)
        {
            // node_f reused as depth scratch, parent as ancestor scratch
#pragma unroll
            for (int r = 0; r < 8; ++r)
            {
                const uint32_t v = lane + 64 * r;
                if (v < nodes)
                {
                    S.node_f[v] = dep[r];
                    S.parent[v] = (uint16_t) anc[r];
                }
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 8; ++r)
            {
                const uint32_t v = lane + 64 * r;
                if (v < nodes && anc[r] != 0xFFFF)
                {
                    dep[r] += S.node_f[anc[r]];
                    anc[r] = S.parent[anc[r]];
                }
            }
            __syncthreads();
        }
        // lengths per symbol
        if (lane < 65)
            for (int i = lane; i < 260; i += 64)
                S.cnt[i] = 0;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; ++r)
        {
            const uint32_t v = lane + 64 * r;
            if (v < nodes)
                S.node_f[v] = dep[r];
        }
        __syncthreads();
        {
            uint32_t id = ex;
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                uint32_t L = 0;
                if (h[r])
                {
                    const uint32_t d = S.node_f[id++];
                    L                = (leaves == 1) ? 1 : (d & 0xFF);
                }
                S.len_s[lane * 4 + r] = (uint8_t) L;
                if (L)
                    atomicAdd(&S.cnt[L], 1u);
            }
        }
        __syncthreads();
        uint64_t bits = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            bits += (uint64_t) h[r] * S.len_s[lane * 4 + r];
        for (int d = 32; d > 0; d >>= 1)
            bits += shfl_xor64(bits, d);
        // canonical codes (:227-261) in uint32 with wrap: first code of length l =
        // sum_{k < l} cnt[k] << (l - k) (terms shifted by >= 32 vanish), then each symbol adds its
        // rank among the symbols of its length (symbol order); one ballot round per distinct length
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t l = (uint32_t) lane * 4 + r + 1;
            uint32_t       c = 0;
            for (uint32_t k = l > 32 ? l - 31 : 1; k < l; ++k)
                c += S.cnt[k] << (l - k);
            S.next[l] = c;
        }
        __syncthreads();
        {
            uint32_t L[4], code[4] = {0, 0, 0, 0};
            bool     todo[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                L[r]    = S.len_s[lane * 4 + r];
                todo[r] = L[r] != 0;
            }
            const uint64_t below = (1ull << lane) - 1ull;
            for (;;)
            {
                const uint32_t cand = todo[0] ? L[0] : todo[1] ? L[1] : todo[2] ? L[2] : todo[3] ? L[3] : 0u;
                const uint64_t any  = __builtin_amdgcn_ballot_w64(cand != 0);
                if (!any)
                    break;
                const uint32_t L0 = __builtin_amdgcn_readlane(cand, (uint32_t) __builtin_ctzll(any));
                uint32_t       before = 0, own = 0;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    before += (uint32_t) __builtin_popcountll(__builtin_amdgcn_ballot_w64(L[r] == L0) & below);
                const uint32_t first = S.next[L0];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (L[r] == L0)
                    {
                        code[r] = first + before + own++;
                        todo[r] = false;
                    }
            }
            reinterpret_cast<uint4*>(codes + (size_t) b * 256)[lane] = make_uint4(code[0], code[1], code[2], code[3]);
        }
        if (lane == 0)
        {
            HuffMetaRec& M  = meta[b];
            M.orig_size     = rle_size[b];
            const uint32_t bc = (uint32_t) bits;  // bra_huffman.c:390-392 accumulates in uint32
            M.encoded_size  = (bc + 7u) / 8u;
        }
        for (int i = lane; i < 256; i += 64)
            meta[b].lengths[i] = S.len_s[i];
        __syncthreads();
    }
}

__global__ void __launch_bounds__(TPB) k_huff_offsets(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, uint64_t* __restrict__ off)
{
    __shared__ uint64_t tmp[8];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0)
        carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nblocks; base += TPB)
    {
        const uint32_t b = base + threadIdx.x;
        const uint64_t v = b < nblocks ? meta[b].encoded_size : 0;
        uint64_t       total;
        const uint64_t ex = block256_exclusive_sum64(v, tmp, &total);
        if (b < nblocks)
            off[b] = carry + ex;
        __syncthreads();
        if (threadIdx.x == 0)
            carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0)
        off[nblocks] = carry;
}

// tiles over the RLE-output CAPACITY of each block; a tile beyond the block's RLE size is empty
// The 16 symbols [i0, i0 + 16) of a tile (one 16-byte load when the tile is full and aligned;
// symbols at or beyond cnt read as 0).
__device__ __forceinline__ void load_syms(const uint8_t* __restrict__ p, uint32_t cnt, uint32_t i0, uint8_t (&sym)[16])
{
    if (i0 + 16 <= cnt && (((uintptr_t) (p + i0)) & 15) == 0)
    {
        const uint4    v    = *reinterpret_cast<const uint4*>(p + i0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k)
            sym[k] = (uint8_t) (w[k >> 2] >> (8 * (k & 3)));
    }
    else
    {
#pragma unroll
        for (int k = 0; k < 16; ++k)
            sym[k] = (i0 + k < cnt) ? p[i0 + k] : 0;
    }
}

__global__ void __launch_bounds__(TPB) k_huff_tilebits(const uint8_t* __restrict__ rle, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                       const HuffMetaRec* __restrict__ meta, uint32_t* __restrict__ tbits)
{
    __shared__ uint8_t  L[256];
    __shared__ uint32_t tmp[8];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const Piece    P    = tiles[t];
        const uint32_t rs   = meta[P.block].orig_size;
        L[threadIdx.x]      = meta[P.block].lengths[threadIdx.x];
        __syncthreads();
        const uint32_t cnt = P.start < rs ? min(P.len, rs - P.start) : 0;
        uint32_t       acc = 0;
        uint8_t        sym[16];
        load_syms(rle + P.off, cnt, threadIdx.x * 16, sym);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            acc += (threadIdx.x * 16 + k < cnt) ? L[sym[k]] : 0u;
        uint32_t total;
        block256_exclusive_sum(acc, tmp, &total);
        if (threadIdx.x == 0)
            tbits[t] = total;
        __syncthreads();
    }
}

// One wave per block: exclusive scan of the tiles' bit counts (64 tiles per step).
__global__ void __launch_bounds__(64) k_huff_tilescan(const uint32_t* __restrict__ first, const uint32_t* __restrict__ count, uint32_t nblocks,
                                                      const uint64_t* __restrict__ payload_off, uint32_t* __restrict__ tbits,
                                                      uint64_t* __restrict__ tbit0)
{
    const int lane = lane_id();
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        uint64_t       run = payload_off[b] * 8;
        const uint32_t t0 = first[b], nt = count[b];
        for (uint32_t c = 0; c < nt; c += 64)
        {
            const uint32_t i   = c + lane;
            const uint32_t v   = i < nt ? tbits[t0 + i] : 0u;
            const uint32_t inc = wave_scan<true>(v, 0u, OpAdd());  // a tile holds < 2^27 bits: 64 of them fit 32 bits
            if (i < nt)
                tbit0[t0 + i] = run + inc - v;
            run += __builtin_amdgcn_readlane(inc, 63);
        }
    }
}

__global__ void k_huff_zero(const uint32_t* __restrict__ tbits, const uint64_t* __restrict__ tbit0, uint32_t ntiles,
                            uint32_t* __restrict__ out_words)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += gridDim.x * blockDim.x)
    {
        if (!tbits[t])
            continue;
        const uint64_t b0 = tbit0[t], b1 = b0 + tbits[t] - 1;
        out_words[b0 >> 5] = 0;
        out_words[b1 >> 5] = 0;
    }
}

__device__ __forceinline__ void or_bits(uint32_t* w, uint64_t pos, uint32_t v, uint32_t nb, bool global)
{
    // place the nb-bit value v at stream bit pos (MSB-first within 32-bit words)
    const uint32_t word = (uint32_t) (pos >> 5), off = (uint32_t) (pos & 31);
    if (off + nb <= 32)
    {
        const uint32_t x = v << (32 - off - nb);
        if (x)
            global ? atomicOr(&w[word], __builtin_bswap32(x)) : atomicOr(&w[word], x);
    }
    else
    {
        const uint32_t spill = off + nb - 32;
        const uint32_t x0    = v >> spill;
        const uint32_t x1    = v << (32 - spill);
        if (x0)
            global ? atomicOr(&w[word], __builtin_bswap32(x0)) : atomicOr(&w[word], x0);
        if (x1)
            global ? atomicOr(&w[word + 1], __builtin_bswap32(x1)) : atomicOr(&w[word + 1], x1);
    }
}

constexpr uint32_t PACK_WORDS = RLE_TILE + 2;  // 32 bits/symbol max on the LDS path

__global__ void __launch_bounds__(TPB) k_huff_pack(const uint8_t* __restrict__ rle, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                   const HuffMetaRec* __restrict__ meta, const uint32_t* __restrict__ codes,
                                                   const uint32_t* __restrict__ tbits, const uint64_t* __restrict__ tbit0,
                                                   uint32_t* __restrict__ out_words)
{
    __shared__ uint2    LC[256];  // (code, length) per symbol: one LDS read per symbol
    __shared__ uint32_t tmp[8];
    __shared__ uint32_t img[PACK_WORDS];
    constexpr int       PT = RLE_TILE / TPB;
    const XcdTiles X = xcd_tiles(ntiles);  // the boundary words two tiles OR into stay in one L2
    for (uint32_t t = X.t; t < X.end; t += X.step)
    {
        const uint32_t nbits = tbits[t];
        if (nbits == 0)
            continue;  // uniform
        const Piece    P  = tiles[t];
        const uint32_t rs = meta[P.block].orig_size;
        LC[threadIdx.x]   = make_uint2(codes[(size_t) P.block * 256 + threadIdx.x], meta[P.block].lengths[threadIdx.x]);
        const uint32_t cnt = min(P.len, rs - P.start);
        const uint64_t g0  = tbit0[t];
        const uint32_t sh  = (uint32_t) (g0 & 31);
        const uint32_t nw  = (sh + nbits + 31) >> 5;
        const bool     lds = nw <= PACK_WORDS;
        if (lds)
            for (uint32_t i = threadIdx.x; i < nw; i += TPB)
                img[i] = 0;
        __syncthreads();
        // this thread's contiguous symbols
        static_assert(PT == 16, "16 symbols per thread");
        const uint32_t i0 = threadIdx.x * PT;
        uint8_t        sym[PT];
        uint2          e[PT];  // code, length of each symbol (read once, kept across the scan's barrier)
        uint32_t       mybits = 0;
        load_syms(rle + P.off, cnt, i0, sym);
#pragma unroll
        for (int k = 0; k < PT; ++k)
        {
            e[k] = (i0 + k < cnt) ? LC[sym[k]] : make_uint2(0, 0);
            mybits += e[k].y;
        }
        if (!lds)
        {
            // global path (codes > 32 bits make the tile image too large for LDS): the words strictly
            // inside the tile are owned by it; zero them before OR-ing (boundary words: k_huff_zero)
            uint32_t* gw = out_words + (g0 >> 5);
            for (uint32_t i = 1 + threadIdx.x; i + 1 < nw; i += TPB)
                gw[i] = 0;
        }
        const uint32_t ex  = block256_exclusive_sum(mybits, tmp);  // (contains __syncthreads)
        uint64_t       pos = lds ? (uint64_t) sh + ex : g0 + ex;
        if (lds)
        {
            // the thread's bits are contiguous: gather them in a 64-bit register and store whole
            // words; only the first and the last word can be shared with a neighbour (atomicOr)
            uint32_t word = (uint32_t) (pos >> 5), nacc = (uint32_t) (pos & 31);
            uint64_t acc   = 0;  // pending bits, MSB-first from bit 63; the first nacc are the neighbour's
            bool     first = true;
            const auto flush = [&]() {
                while (nacc >= 32)
                {
                    const uint32_t v = (uint32_t) (acc >> 32);
                    if (first)
                    {
                        if (v)
                            atomicOr(&img[word], v);
                        first = false;
                    }
                    else
                        img[word] = v;
                    acc <<= 32;
                    nacc -= 32;
                    ++word;
                }
            };
#pragma unroll
            for (int k = 0; k < PT; ++k)
            {
                if (i0 + k >= cnt)
                    continue;  // (not break: the loop must unroll fully to keep e[] in registers)
                uint32_t nb = e[k].y;
                if (nb > 32)
                {
                    nacc += nb - 32;  // leading zero bits of a wrapped long code
                    flush();
                    nb = 32;
                }
                acc |= ((uint64_t) e[k].x << (64 - nb)) >> nacc;
                nacc += nb;
                flush();
            }
            if (nacc && (uint32_t) (acc >> 32))
                atomicOr(&img[word], (uint32_t) (acc >> 32));
        }
        else
        {
#pragma unroll
            for (int k = 0; k < PT; ++k)
            {
                if (i0 + k >= cnt)
                    continue;
                uint32_t       nb = e[k].y;
                const uint32_t c  = e[k].x;
                if (nb > 32)
                {
                    pos += nb - 32;  // leading zero bits of a wrapped long code
                    nb = 32;
                }
                or_bits(out_words, pos, c, nb, true);
                pos += nb;
            }
        }
        __syncthreads();
        if (lds)
        {
            uint32_t* gw = out_words + (g0 >> 5);
            for (uint32_t i = threadIdx.x; i < nw; i += TPB)
            {
                const uint32_t v = __builtin_bswap32(img[i]);
                if (i == 0 || i == nw - 1)
                {
                    if (v)
                        atomicOr(&gw[i], v);
                }
                else
                    gw[i] = v;
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// decode
// ------------------------------------------------------------------------------------------------
constexpr uint32_t TREE_CAP = 256 * 256 + 4;  // nodes per block (a code inserts <= len nodes)
constexpr int      PEEK     = 11;

// Reference tree from lengths (bra_huffman.c:263-348), one thread per block.  child[2*v+bit],
// -1 = none.  status[b] = 1 on a failed insertion (the reference returns NULL).
__global__ void k_huff_tree(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, int32_t* __restrict__ child, uint8_t* __restrict__ sym,
                            uint32_t* __restrict__ status)
{
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += gridDim.x * blockDim.x)
    {
        const HuffMetaRec& M  = meta[b];
        int32_t*           ch = child + (size_t) b * TREE_CAP * 2;
        uint8_t*           sy = sym + (size_t) b * TREE_CAP;
        uint32_t           count[257] = {0};
        for (int s = 0; s < 256; ++s)
            if (M.lengths[s])
                count[M.lengths[s]]++;
        uint32_t next[257];
        uint32_t code = 0;
        for (int l = 1; l <= 256; ++l)
        {
            code <<= 1;
            next[l] = code;
            code += count[l];
        }
        uint32_t nodes = 1;
        ch[0] = ch[1] = -1;
        sy[0]         = 0;
        uint32_t st   = 0;
        for (int s = 0; s < 256 && !st; ++s)
        {
            const uint32_t l = M.lengths[s];
            if (!l)
                continue;
            const uint32_t c   = next[l]++;
            uint32_t       cur = 0;
            for (uint32_t j = 0; j < l; ++j)
            {
                const uint32_t bi  = l - 1 - j;
                const int      bit = bi < 32 ? (int) ((c >> bi) & 1u) : 0;
                if (j == l - 1)
                {
                    if (ch[2 * cur + bit] != -1)
                    {
                        st = 1;
                        break;
                    }
                    ch[2 * cur + bit] = (int32_t) nodes;
                    ch[2 * nodes] = ch[2 * nodes + 1] = -1;
                    sy[nodes++]                       = (uint8_t) s;
                }
                else
                {
                    if (ch[2 * cur + bit] == -1)
                    {
                        ch[2 * cur + bit] = (int32_t) nodes;
                        ch[2 * nodes] = ch[2 * nodes + 1] = -1;
                        sy[nodes++]                       = 0;
                    }
                    cur = (uint32_t) ch[2 * cur + bit];
                }
            }
        }
        status[b] = st;
    }
}

// 11-bit primary table per block: entry = kind(2) | used(4) | value(24)
//   kind 0: leaf `value` reached after `used` bits; kind 1: continue at node `value` after 11 bits;
//   kind 2: dead edge (decode error) after `used` bits.
__global__ void k_huff_table(const int32_t* __restrict__ child, const uint8_t* __restrict__ sym, uint32_t nblocks, uint32_t* __restrict__ table)
{
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const int32_t* ch = child + (size_t) b * TREE_CAP * 2;
        for (uint32_t v = threadIdx.x; v < (1u << PEEK); v += blockDim.x)
        {
            uint32_t cur = 0, e = 0;
            int      j   = 0;
            for (; j < PEEK; ++j)
            {
                const int bit = (v >> (PEEK - 1 - j)) & 1;
                const int nx  = ch[2 * cur + bit];
                if (nx < 0)
                {
                    e = (2u << 28) | ((uint32_t) (j + 1) << 24);
                    break;
                }
                cur = (uint32_t) nx;
                if (ch[2 * cur] < 0 && ch[2 * cur + 1] < 0)
                {
                    e = (0u << 28) | ((uint32_t) (j + 1) << 24) | sym[(size_t) b * TREE_CAP + cur];
                    break;
                }
            }
            if (j == PEEK)
                e = (1u << 28) | ((uint32_t) PEEK << 24) | cur;
            table[(size_t) b * (1u << PEEK) + v] = e;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Segment-parallel decode (self-synchronisation).  A block's bit stream is cut into SEG_BITS-bit
// segments.  Pass 1 decodes every segment speculatively from its first bit up to the first
// codeword boundary at or past its end.  Pass 2 restarts each segment from the previous segment's
// exit (the true boundary) and walks the speculative path alongside until the two meet (Huffman
// codes resynchronise within a few codewords): the counts after the meeting point are reused.  A
// segment whose true path does not meet changes its exit, so pass 2 repeats until no exit moves.
// Pass 3 prefix-sums the symbol counts per block, pass 4 decodes each segment's true path into
// its output range, and a per-block pass applies the reference's end-of-stream rules (decode stops
// at orig_size; a stream that ends early or holds a dead edge before it is rejected; :455-498).
// ------------------------------------------------------------------------------------------------
constexpr uint32_t SEG_BITS = 2048;

__device__ __forceinline__ uint32_t hd_peek(const uint8_t* __restrict__ src, uint32_t nbytes, uint64_t p, int n)
{
    const uint32_t byt = (uint32_t) (p >> 3);
    uint64_t       w;
    if (byt + 8 <= nbytes)
    {
        const uintptr_t a  = (uintptr_t) (src + byt);
        const uint64_t* q  = (const uint64_t*) (a & ~(uintptr_t) 7);
        const uint32_t  sh = (uint32_t) (a & 7) * 8;
        const uint64_t  lo = q[0];
        const uint64_t  x  = sh ? (lo >> sh) | (q[1] << (64 - sh)) : lo;  // q[1] holds byte byt + 7 < nbytes
        w                  = __builtin_bswap64(x);
    }
    else
    {
        w = 0;
        for (int i = 0; i < 8; ++i)
            w = (w << 8) | (byt + i < nbytes ? src[byt + i] : 0);
    }
    return (uint32_t) ((w << (p & 7)) >> (64 - n));
}

struct HdBlock
{
    const uint8_t*  src;
    uint32_t        nbytes;
    uint64_t        nbits;
    const uint32_t* tb;
    const int32_t*  ch;
    const uint8_t*  sy;
};

__device__ __forceinline__ HdBlock hd_block(const HuffMetaRec* meta, const uint8_t* payload, const uint64_t* payload_off, const int32_t* child,
                                            const uint8_t* sym, const uint32_t* table, uint32_t b)
{
    HdBlock B;
    B.src    = payload + payload_off[b];
    B.nbytes = meta[b].encoded_size;
    B.nbits  = (uint64_t) B.nbytes * 8;
    B.tb     = table + (size_t) b * (1u << PEEK);
    B.ch     = child + (size_t) b * TREE_CAP * 2;
    B.sy     = sym + (size_t) b * TREE_CAP;
    return B;
}

// One codeword at pos (the reference's walk, :455-482, through the 11-bit table): true and the
// symbol, or false on a dead edge / the end of the data.
__device__ __forceinline__ bool hd_step(const HdBlock& B, uint64_t& pos, uint32_t& sym)
{
    if (pos >= B.nbits)
        return false;
    const uint32_t e    = B.tb[hd_peek(B.src, B.nbytes, pos, PEEK)];
    const uint32_t kind = e >> 28, used = (e >> 24) & 15;
    if (pos + used > B.nbits || kind == 1)
    {
        uint32_t cur = 0;
        if (!(pos + used > B.nbits))
        {
            cur = e & 0xFFFFFF;
            pos += PEEK;
        }
        while (pos < B.nbits)
        {
            const int nx = B.ch[2 * cur + (int) hd_peek(B.src, B.nbytes, pos, 1)];
            ++pos;
            if (nx < 0)
                return false;
            cur = (uint32_t) nx;
            if (B.ch[2 * cur] < 0 && B.ch[2 * cur + 1] < 0)
            {
                sym = B.sy[cur];
                return true;
            }
        }
        return false;
    }
    if (kind == 2)
        return false;
    sym = e & 0xFFFFFF;
    pos += used;
    return true;
}

struct HdSeg
{
    uint32_t exit;   // bit position of the first codeword boundary at or past the segment end
    uint32_t cnt;    // symbols decoded in the segment
    uint32_t start;  // true start (pass 2)
    uint32_t bad;    // the path met a dead edge / the end of the data
};

__device__ __forceinline__ uint32_t hd_seg_block(const uint32_t* __restrict__ seg_base, uint32_t nblocks, uint32_t g)
{
    uint32_t lo = 0, hi = nblocks;  // last b with seg_base[b] <= g
    while (hi - lo > 1)
    {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg_base[mid] <= g)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

__global__ void k_hd_spec(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, const uint8_t* __restrict__ payload,
                          const uint64_t* __restrict__ payload_off, const int32_t* __restrict__ child, const uint8_t* __restrict__ sym,
                          const uint32_t* __restrict__ table, const uint32_t* __restrict__ tree_status, const uint32_t* __restrict__ seg_base,
                          uint32_t nseg, HdSeg* __restrict__ seg)
{
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nseg; g += gridDim.x * blockDim.x)
    {
        const uint32_t b = hd_seg_block(seg_base, nblocks, g), j = g - seg_base[b];
        HdSeg          S{0, 0, 0, 1};
        if (!tree_status[b])
        {
            const HdBlock  B   = hd_block(meta, payload, payload_off, child, sym, table, b);
            const uint64_t end = min((uint64_t) (j + 1) * SEG_BITS, B.nbits);
            uint64_t       pos = (uint64_t) j * SEG_BITS;
            uint32_t       cnt = 0, sy;
            bool           ok  = true;
            while (pos < end && (ok = hd_step(B, pos, sy)))
                ++cnt;
            S = HdSeg{(uint32_t) pos, cnt, (uint32_t) ((uint64_t) j * SEG_BITS), ok ? 0u : 1u};
        }
        seg[g] = S;
    }
}

// Pass 2: cur[] -> nxt[]; *changed is set when a segment's exit moved.
__global__ void k_hd_sync(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, const uint8_t* __restrict__ payload,
                          const uint64_t* __restrict__ payload_off, const int32_t* __restrict__ child, const uint8_t* __restrict__ sym,
                          const uint32_t* __restrict__ table, const uint32_t* __restrict__ tree_status, const uint32_t* __restrict__ seg_base,
                          uint32_t nseg, const HdSeg* __restrict__ spec, const HdSeg* __restrict__ cur, HdSeg* __restrict__ nxt,
                          uint32_t* __restrict__ changed)
{
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nseg; g += gridDim.x * blockDim.x)
    {
        const uint32_t b = hd_seg_block(seg_base, nblocks, g), j = g - seg_base[b];
        if (j == 0 || tree_status[b])
        {
            nxt[g] = cur[g];
            continue;
        }
        const HdSeg P = cur[g - 1];
        HdSeg       R;
        if (P.bad)
            R = HdSeg{P.exit, 0, P.exit, 1};  // the true path already failed: nothing here counts
        else
        {
            const HdBlock  B   = hd_block(meta, payload, payload_off, child, sym, table, b);
            const uint64_t end = min((uint64_t) (j + 1) * SEG_BITS, B.nbits);
            const HdSeg    Sp  = spec[g];
            uint64_t       a = P.exit, q = (uint64_t) j * SEG_BITS;
            uint32_t       ca = 0, cq = 0, sy;
            bool           aok = true, qok = true, synced = false;
            while (aok && a < end)
            {
                if (a == q && qok)
                {
                    synced = true;
                    break;
                }
                if (qok && q < a)
                {
                    if (hd_step(B, q, sy))
                        ++cq;
                    else
                        qok = false;
                }
                else if ((aok = hd_step(B, a, sy)))
                    ++ca;
            }
            if (synced)
                R = HdSeg{Sp.exit, Sp.cnt - cq + ca, (uint32_t) P.exit, Sp.bad};
            else
                R = HdSeg{(uint32_t) a, ca, (uint32_t) P.exit, aok ? 0u : 1u};
        }
        if (R.exit != cur[g].exit || R.bad != cur[g].bad)  // what the next segment starts from
            atomicExch(changed, 1u);
        nxt[g] = R;
    }
}

// Pass 3: per block, exclusive prefix of the symbol counts; status for failures before orig_size.
__global__ void __launch_bounds__(256) k_hd_prefix(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, const uint32_t* __restrict__ tree_status,
                                                   const uint32_t* __restrict__ seg_base, const HdSeg* __restrict__ seg, uint32_t* __restrict__ off,
                                                   uint32_t* __restrict__ status)
{
    __shared__ uint32_t tmp[8];
    __shared__ uint32_t fail;
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t g0 = seg_base[b], n = seg_base[b + 1] - g0, osz = meta[b].orig_size;
        if (threadIdx.x == 0)
            fail = tree_status[b] ? 1u : 0u;
        __syncthreads();
        uint32_t run = 0;
        for (uint32_t i0 = 0; i0 < n; i0 += 256)
        {
            const uint32_t i   = i0 + threadIdx.x;
            const HdSeg    S   = i < n ? seg[g0 + i] : HdSeg{0, 0, 0, 0};
            uint32_t       tot;
            const uint32_t ex  = block256_exclusive_sum(S.cnt, tmp, &tot);
            if (i < n)
            {
                off[g0 + i] = run + ex;
                if (S.bad && run + ex + S.cnt < osz)
                    atomicExch(&fail, 1u);  // the true path dies before symbol orig_size
            }
            run += tot;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            status[b] = (fail || run < osz) ? 1u : 0u;  // ran out of data before orig_size symbols
        __syncthreads();
    }
}

// Pass 4: decode each segment's true path into out[off, off + cnt), clipped at orig_size; the
// segment holding symbol orig_size - 1 records where it ends.
__global__ void k_hd_write(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, const uint8_t* __restrict__ payload,
                           const uint64_t* __restrict__ payload_off, const int32_t* __restrict__ child, const uint8_t* __restrict__ sym,
                           const uint32_t* __restrict__ table, const uint32_t* __restrict__ status, const uint32_t* __restrict__ seg_base,
                           uint32_t nseg, const HdSeg* __restrict__ seg, const uint32_t* __restrict__ off, uint8_t* __restrict__ out,
                           const uint64_t* __restrict__ out_base, uint64_t* __restrict__ end_pos)
{
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nseg; g += gridDim.x * blockDim.x)
    {
        const uint32_t b = hd_seg_block(seg_base, nblocks, g);
        if (status[b])
            continue;
        const HdSeg    S   = seg[g];
        const uint32_t osz = meta[b].orig_size, o = off[g];
        if (o >= osz || S.cnt == 0)
            continue;
        const HdBlock  B   = hd_block(meta, payload, payload_off, child, sym, table, b);
        uint8_t*       dst = out + out_base[b];
        uint64_t       pos = S.start;
        const uint32_t n   = min(S.cnt, osz - o);
        uint32_t       sy  = 0;
        for (uint32_t i = 0; i < n; ++i)
        {
            (void) hd_step(B, pos, sy);
            dst[o + i] = (uint8_t) sy;
        }
        if (o + n == osz)
            end_pos[b] = pos;
    }
}

// Pass 5: the reference's end-of-stream walk: it leaves the bit loop of the current byte and keeps
// walking the remaining whole bytes; a completed symbol there would overrun its buffer (error), a
// dead edge is an error, an unfinished walk is ignored.
__global__ void k_hd_tail(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, const uint8_t* __restrict__ payload,
                          const uint64_t* __restrict__ payload_off, const int32_t* __restrict__ child, const uint8_t* __restrict__ sym,
                          const uint32_t* __restrict__ table, const uint64_t* __restrict__ end_pos, uint32_t* __restrict__ status)
{
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += gridDim.x * blockDim.x)
    {
        if (status[b])
            continue;
        const HdBlock B   = hd_block(meta, payload, payload_off, child, sym, table, b);
        uint64_t      p2  = meta[b].orig_size ? ((end_pos[b] + 7) & ~7ull) : 0;
        uint32_t      cur = 0, err = 0;
        while (p2 < B.nbits)
        {
            const int nx = B.ch[2 * cur + (int) hd_peek(B.src, B.nbytes, p2, 1)];
            ++p2;
            if (nx < 0)
            {
                err = 1;
                break;
            }
            cur = (uint32_t) nx;
            if (B.ch[2 * cur] < 0 && B.ch[2 * cur + 1] < 0)
            {
                err = 1;
                break;
            }
        }
        status[b] = err;
    }
}

// ------------------------------------------------------------------------------------------------
// Canonical fast path.  A block whose code lengths are "clean" (at least one symbol, every length
// <= 30, Kraft sum <= 1) has a reference tree that is exactly its canonical code: codes are
// prefix-free, so the tree rebuild never collides (bra_huffman.c:263-348) and decoding walks the
// canonical intervals.  Such blocks decode through tables (11-bit primary LUT, left-justified
// interval limits for longer codes) and exact per-segment transfer functions:
//   k_hd_canon   per block: interval limits, symbols by (length, value), the 11-bit LUT;
//   k_hd_trans   per 2048-bit segment (one lane each, the block's tables in LDS, the bits in a
//                4-dword register window): for every possible entry bit offset e < lmax (the true
//                path enters the segment within lmax bits of its start) the exit offset past the
//                segment end, the symbol count and whether the path dies (dead edge / out of data).
//                The path from e = 0 records its codeword boundaries over the first 512 bits; a
//                path from e > 0 that lands on one of them has merged and takes its count from
//                the boundary's rank -- Huffman paths resynchronise within a few codewords, while
//                codes of near-equal lengths (uniform data) keep separate phases and are walked out.
//                No iteration over segments: the round-1 self-synchronisation loop needed up to 31
//                passes on uniform random data (the phases drift).
//   k_hd_chain   per block: follow the true entry from segment to segment -> entry and output
//                offset of every segment, and the reference's acceptance (no death before symbol
//                orig_size, enough data);
//   k_hd_write2  per segment: decode the true path into its output range;
//   k_hd_tail2   per block: the reference's end-of-stream walk (:455-498) on the intervals.
// Any block that is not clean sends the batch to the tree-walking path above.
// ------------------------------------------------------------------------------------------------
// k_hd_trans walks the entries > 0 two at a time (one at a time, or 3 or 4 in lockstep, measured slower)
constexpr uint32_t HD2_SEG   = 2048;  // bits per segment
constexpr uint32_t HD2_LMAX  = 30;
constexpr uint32_t HD2_TPB   = 256;   // k_hd_trans: a lane per segment, HD2_TPB segments per task
constexpr uint32_t HD2_WTPB  = 4 * HD2_TPB;  // k_hd_write2: four lanes per segment
constexpr uint32_t HD2_REFB  = 512;   // boundary bitmap of the reference path (bits from the segment start;
                                      // 64 / 128 / 256 / 512 / 1024: text decode 14.9 / 16.3 / 17.9 / 19.5 / 18.5 GB/s)
constexpr uint32_t HD2_STRD  = 32;    // transfer words per segment
constexpr uint32_t HD2_TAB   = 2304;  // u32 words per block table
constexpr uint32_t HD2_SUB   = HD2_SEG / 4;  // k_hd_write2: four lanes per segment, from sub records
                                             // every HD2_SUB bits of the entry-0 path
static_assert(HD2_REFB <= HD2_SUB, "a path joins the entry-0 path before the first sub record");
static_assert(HD2_LMAX + 2 <= HD2_STRD, "the sub records follow the entries' transfer words");
static_assert(HD2_SEG <= 2048 && HD2_LMAX < 32, "ranks and offsets of the sub records fit 11 + 5 bits");

// table layout (u32 words)
constexpr uint32_t T_LUT = 0, T_LIM = 2048, T_FIRST = 2112, T_IDX = 2144, T_PERM = 2176, T_INFO = 2240;  // info: lmax, clean, even

struct Hd2Lds
{
    uint32_t lut[2048];
    uint64_t lim[32];
    uint32_t first[32];
    uint32_t idx[32];
    uint8_t  perm[256];
    uint32_t lmax;
};

__global__ void __launch_bounds__(256) k_hd_canon(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, uint32_t* __restrict__ tab,
                                                  uint32_t* __restrict__ unclean)
{
    __shared__ uint32_t ln[256], cnt[257];
    __shared__ uint64_t lim[32];
    __shared__ uint32_t first[32], idx[32], sh_lmax, sh_clean, sh_even;
    __shared__ __attribute__((aligned(4))) uint8_t perm[256];
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        uint32_t* T = tab + (size_t) b * HD2_TAB;
        const uint32_t t = threadIdx.x;
        ln[t]   = meta[b].lengths[t];
        cnt[t]  = 0;
        perm[t] = 0;
        if (t == 0)
            cnt[256] = 0;
        __syncthreads();
        if (ln[t])
            atomicAdd(&cnt[ln[t]], 1u);
        __syncthreads();
        if (t == 0)
        {
            uint32_t lmax = 0, lmin = 0, nsym = 0;
            for (uint32_t l = 1; l <= 255; ++l)
                if (cnt[l])
                {
                    lmin = lmin ? lmin : l;
                    lmax = l;
                    nsym += cnt[l];
                }
            // code lengths within 2 of each other (near-uniform data): paths from different entries
            // keep their phases, so k_hd_trans does not try the guessed entries
            sh_even = lmax - lmin <= 2 ? 1u : 0u;
            bool     clean = nsym > 0 && lmax <= HD2_LMAX;
            uint64_t code = 0;
            uint32_t id   = 0;
            for (uint32_t l = 1; l < 32; ++l)
            {
                code <<= 1;
                const uint32_t c = l <= HD2_LMAX ? cnt[l] : 0u;
                first[l]         = (uint32_t) code;
                idx[l]           = id;
                code += c;
                id += c;
                lim[l] = code << (32 - l);  // left-justified end of the length-l interval
            }
            first[0] = idx[0] = 0;
            lim[0]            = 0;
            clean             = clean && lim[lmax < 32 ? lmax : 31] <= (1ull << 32);  // Kraft sum <= 1
            sh_lmax           = lmax;
            sh_clean          = clean ? 1u : 0u;
            if (!clean)
                atomicOr(unclean, 1u);
        }
        __syncthreads();
        const uint32_t lmax = sh_lmax;
        if (sh_clean)
        {
            // symbols by (length, value)
            if (ln[t])
            {
                uint32_t r = 0;
                for (uint32_t u = 0; u < t; ++u)
                    r += ln[u] == ln[t] ? 1u : 0u;
                perm[idx[ln[t]] + r] = (uint8_t) t;
            }
            __syncthreads();
            // 11-bit LUT: sym | len << 8 | kind << 13 (0 leaf, 1 longer code, 2 dead)
            for (uint32_t v = t; v < 2048; v += 256)
            {
                const uint64_t vj    = (uint64_t) v << 21;
                uint32_t       e     = 2u << 13;
                bool           found = false;
                for (uint32_t l = 1; l <= min(lmax, 11u) && !found; ++l)
                    if (vj < lim[l])
                    {
                        e     = perm[idx[l] + (uint32_t) (v >> (11 - l)) - first[l]] | (l << 8);
                        found = true;
                    }
                if (!found && lmax > 11 && vj < lim[lmax])
                    e = 1u << 13;
                T[T_LUT + v] = e;
            }
            if (t < 32)
            {
                reinterpret_cast<uint64_t*>(T + T_LIM)[t] = lim[t];
                T[T_FIRST + t]                            = first[t];
                T[T_IDX + t]                              = idx[t];
            }
            if (t < 64)
                T[T_PERM + t] = reinterpret_cast<const uint32_t*>(perm)[t];
            if (t == 0)
            {
                T[T_INFO]     = lmax;
                T[T_INFO + 1] = 1;
                T[T_INFO + 2] = sh_even;
            }
        }
        else if (t == 0)
        {
            T[T_INFO]     = lmax;
            T[T_INFO + 1] = 0;
        }
        __syncthreads();
    }
}

__device__ __forceinline__ void hd2_load_tables(const uint32_t* __restrict__ T, Hd2Lds& L)
{
    for (uint32_t i = threadIdx.x; i < 2048; i += blockDim.x)
        L.lut[i] = T[T_LUT + i];
    if (threadIdx.x < 32)
    {
        L.lim[threadIdx.x]   = reinterpret_cast<const uint64_t*>(T + T_LIM)[threadIdx.x];
        L.first[threadIdx.x] = T[T_FIRST + threadIdx.x];
        L.idx[threadIdx.x]   = T[T_IDX + threadIdx.x];
    }
    if (threadIdx.x < 64)
        reinterpret_cast<uint32_t*>(L.perm)[threadIdx.x] = T[T_PERM + threadIdx.x];
    if (threadIdx.x == 0)
        L.lmax = T[T_INFO];
    __syncthreads();
}

// One codeword from the left-justified 32 bits v and its primary LUT entry e = L.lut[v >> 21]:
// length and symbol, false on a dead edge.
__device__ __forceinline__ bool hd2_dec_e(const Hd2Lds& L, uint32_t v, uint32_t e, uint32_t& len, uint32_t& sym)
{
    const uint32_t kind = e >> 13;
    if (kind == 0)
    {
        len = (e >> 8) & 31u;
        sym = e & 0xFFu;
        return true;
    }
    if (kind == 2)
        return false;
    for (uint32_t l = 12; l <= L.lmax; ++l)
        if ((uint64_t) v < L.lim[l])
        {
            len = l;
            sym = L.perm[L.idx[l] + (v >> (32 - l)) - L.first[l]];
            return true;
        }
    return false;
}

// One codeword from the left-justified 32 bits v: length and symbol, false on a dead edge.
__device__ __forceinline__ bool hd2_dec(const Hd2Lds& L, uint32_t v, uint32_t& len, uint32_t& sym)
{
    return hd2_dec_e(L, v, L.lut[v >> 21], len, sym);
}

// The bits of one block seen through a 4-dword window (MSB-first, byte-swapped dwords).  Block bit p
// is bit q = p + lead of the dword-aligned stream starting at `base`; dwords past the block's data
// are clamped to its last dword (their bits are never decisive: a codeword that needs them does
// not fit in the data).
struct BitWin
{
    const uint32_t* base;
    uint32_t        lead, kmax;
    uint32_t        wb;  // bit q of W[0]'s first bit
    uint32_t        W[4];

    __device__ __forceinline__ uint32_t ld(uint32_t k) const { return __builtin_bswap32(base[min(k, kmax)]); }
    __device__ __forceinline__ void     init(uint32_t p)
    {
        const uint32_t q = p + lead;
        wb               = q & ~31u;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            W[i] = ld((wb >> 5) + i);
    }
    __device__ __forceinline__ uint32_t peek(uint32_t p)
    {
        uint32_t o = p + lead - wb;
        if (o >= 64)
        {
            W[0] = W[1];
            W[1] = W[2];
            W[2] = W[3];
            wb += 32;
            W[3] = ld((wb >> 5) + 3);
            o -= 32;
        }
        // o < 64 here (a codeword moves p by <= 30 bits): dword o >> 5 is W[0] or W[1]; the choice
        // is made with masks (a select chain was turned into an indexed scratch load)
        const uint32_t m = 0u - (o >> 5), sh = o & 31;
        const uint32_t a = W[0] ^ ((W[0] ^ W[1]) & m);
        const uint32_t c = W[1] ^ ((W[1] ^ W[2]) & m);
        return (uint32_t) ((((uint64_t) a << 32) | c) >> (32 - sh));
    }
};

__device__ __forceinline__ BitWin hd2_win(const uint8_t* payload, uint64_t off, uint32_t nbytes)
{
    BitWin         W;
    const uint64_t a = (uint64_t) (uintptr_t) (payload + off);
    W.base           = reinterpret_cast<const uint32_t*>((uintptr_t) (a & ~3ull));
    W.lead           = (uint32_t) (a & 3) * 8;
    W.kmax           = nbytes ? (uint32_t) ((a & 3) + nbytes - 1) >> 2 : 0u;
    W.wb             = 0;
    return W;
}

struct Hd2Task
{
    uint32_t block, seg0;
};

constexpr uint32_t HD2_UNSET = 0xFFFFFFFFu;  // a transfer word not computed (real words have bits 21-29 clear)

// Walks of entries ea (and eb when `two`) of segment [s, stop) until they end, die or land on a
// codeword start of the entry-0 path (boundary bitmap bm over its first HD2_REFB bits; r0 / c0:
// its transfer word without the count, and its count).  Two walks in lockstep: both paths' window
// loads and LUT reads are issued before either result is used (one path's step is a dependent
// load chain).
__device__ __forceinline__ void hd2_walk_entries(const Hd2Lds& L, const uint8_t* payload, uint64_t off, uint32_t nbytes, uint32_t s, uint32_t stop,
                                                 const uint32_t (&bm)[HD2_REFB / 32], uint32_t r0, uint32_t c0, uint32_t ea, uint32_t eb,
                                                 bool two, uint32_t& ra, uint32_t& rb, bool give_up = false)
{
    const uint32_t nbits = nbytes * 8;
    BitWin         WA = hd2_win(payload, off, nbytes), WB = hd2_win(payload, off, nbytes);
    uint32_t       pa = s + ea, pb = s + (two ? eb : ea), ca = 0, cb = 0;
    bool           la = true, lb = two;
    ra = rb = 0;
    WA.init(pa);
    WB.init(pb);
    // end / merge checks of one path (registers only)
    const auto check = [&](uint32_t pq, uint32_t cq, uint32_t& rq, bool& lq) __attribute__((always_inline)) {
        if (!lq)
            return;
        if (pq >= stop)
        {
            rq = (((pq - stop) & 31u) << 16) | cq;
            lq = false;
            return;
        }
        const uint32_t d = pq - s;
        if (give_up && d >= HD2_REFB)
        {
            // past the bitmap the path can no longer join: leave it to HD_REST
            rq = HD2_UNSET;
            lq = false;
            return;
        }
        if (d < HD2_REFB)
        {
            uint32_t wsel = 0;
#pragma unroll
            for (int i = 0; i < (int) (HD2_REFB / 32); ++i)
                wsel = (d >> 5) == (uint32_t) i ? bm[i] : wsel;
            if ((wsel >> (d & 31)) & 1u)
            {
                uint32_t rank = 0;
#pragma unroll
                for (int i = 0; i < (int) (HD2_REFB / 32); ++i)
                {
                    const uint32_t m = (d >> 5) == (uint32_t) i ? ((1u << (d & 31)) - 1u) : ((d >> 5) > (uint32_t) i ? 0xFFFFFFFFu : 0u);
                    rank += (uint32_t) __popc(bm[i] & m);
                }
                rq = r0 | (cq + c0 - rank);
                lq = false;
            }
        }
    };
    const auto advance = [&](uint32_t v, uint32_t le, uint32_t& pq, uint32_t& cq, uint32_t& rq, bool& lq) __attribute__((always_inline)) {
        if (!lq)
            return;
        uint32_t len, sym;
        if (!hd2_dec_e(L, v, le, len, sym) || len > nbits - pq)
        {
            rq = (1u << 31) | (((pq - stop) & 31u) << 16) | cq;
            lq = false;
            return;
        }
        pq += len;
        ++cq;
    };
    while (la || lb)
    {
        check(pa, ca, ra, la);
        check(pb, cb, rb, lb);
        const uint32_t va = WA.peek(pa), vb = WB.peek(pb);
        const uint32_t xa = L.lut[va >> 21], xb = L.lut[vb >> 21];
        advance(va, xa, pa, ca, ra, la);
        advance(vb, xb, pb, cb, rb, lb);
    }
}

// Transfer words of the segments, in three passes (HD_E0, HD_GUESS, HD_REST):
//   HD_E0     the entry-0 path of every segment: its word (bit 30: "joined the entry-0 path", trivially),
//             the sub records, its boundary bitmap over the first HD2_REFB bits (bmbuf), and
//             HD2_UNSET in the words of the other entries;
//   HD_GUESS  the entry where the entry-0 path of the segment before leaves it (the true entry
//             whenever the true path joined its entry-0 path there; k_hd_chain's guess): that one
//             walk per segment, given up past the bitmap's HD2_REFB bits (it can no longer join).
//             A guess that does not join marks its task and the next one;
//   HD_REST   every other entry, for the marked tasks only.
// Huffman codes of unequal lengths resynchronise within a few codewords, so text-like data needs
// the first two passes only (text: 1.03 -> 0.62 ms); blocks whose code lengths lie within 2 of
// each other (uniform bytes: paths keep their phases) walk every entry in HD_E0, as one pass.
enum : int
{
    HD_E0    = 0,
    HD_GUESS = 1,
    HD_REST  = 2
};

template <int MODE>
__global__ void __launch_bounds__(HD2_TPB) k_hd_trans(const HuffMetaRec* __restrict__ meta, const uint8_t* __restrict__ payload,
                                                      const uint64_t* __restrict__ payload_off, const uint32_t* __restrict__ tab,
                                                      const Hd2Task* __restrict__ tasks, uint32_t ntasks, const uint32_t* __restrict__ seg_base,
                                                      uint32_t* __restrict__ trans, uint32_t* __restrict__ bmbuf, uint32_t* __restrict__ tflag)
{
    __shared__ Hd2Lds L;
    for (uint32_t tk = blockIdx.x; tk < ntasks; tk += gridDim.x)
    {
        if (MODE == HD_REST && tflag[tk] == 0)
            continue;  // uniform over the workgroup
        const Hd2Task  K = tasks[tk];
        const uint32_t b = K.block;
        __syncthreads();
        hd2_load_tables(tab + (size_t) b * HD2_TAB, L);
        const uint32_t nbytes = meta[b].encoded_size, nbits = nbytes * 8;
        const uint32_t j = K.seg0 + threadIdx.x, g0 = seg_base[b], ns = seg_base[b + 1] - g0;
        if (j >= ns)
            continue;
        const uint32_t s = j * HD2_SEG, stop = min(s + HD2_SEG, nbits), nent = j == 0 ? 1u : L.lmax;
        uint32_t*      out = trans + (size_t) (g0 + j) * HD2_STRD;
        uint4*         bmo = reinterpret_cast<uint4*>(bmbuf + (size_t) (g0 + j) * (HD2_REFB / 32));
        uint32_t       bm[HD2_REFB / 32];
        if (MODE == HD_E0)
        {
            // the reference path from entry 0, recording its boundaries over the first HD2_REFB bits
#pragma unroll
            for (int i = 0; i < (int) (HD2_REFB / 32); ++i)
                bm[i] = 0;
            BitWin W = hd2_win(payload, payload_off[b], nbytes);
            W.init(s);
            uint32_t p = s, c = 0, bad = 0, len, sym;
            // the path's first codeword at or after bits HD2_SUB, 2 HD2_SUB, 3 HD2_SUB: (offset past
            // the mark << 11) | rank, 0xFFFF when the path ends before (k_hd_write2 starts its
            // sub-segment lanes there)
            uint32_t mark = HD2_SUB, sub1 = 0xFFFFu, sub2 = 0xFFFFu, sub3 = 0xFFFFu;
            while (p < stop)
            {
                const uint32_t d = p - s;
                if (d < HD2_REFB)
                {
#pragma unroll
                    for (int i = 0; i < (int) (HD2_REFB / 32); ++i)
                        if ((d >> 5) == (uint32_t) i)
                            bm[i] |= 1u << (d & 31);
                }
                if (d >= mark)
                {
                    const uint32_t rec = ((d - mark) << 11) | c;
                    sub1               = mark == HD2_SUB ? rec : sub1;
                    sub2               = mark == 2 * HD2_SUB ? rec : sub2;
                    sub3               = mark == 3 * HD2_SUB ? rec : sub3;
                    mark += HD2_SUB;
                }
                if (!hd2_dec(L, W.peek(p), len, sym) || len > nbits - p)
                {
                    bad = 1;
                    break;
                }
                p += len;
                ++c;
            }
            // bit 30: the path joins the entry-0 path (so k_hd_write2 may split it at the sub records)
            const uint32_t w0 = (bad << 31) | (1u << 30) | (((p - stop) & 31u) << 16) | c;
            uint4*         o4 = reinterpret_cast<uint4*>(out);
            o4[0]             = make_uint4(w0, HD2_UNSET, HD2_UNSET, HD2_UNSET);
#pragma unroll
            for (int i = 1; i < (int) (HD2_STRD / 4) - 1; ++i)
                o4[i] = make_uint4(HD2_UNSET, HD2_UNSET, HD2_UNSET, HD2_UNSET);
            o4[HD2_STRD / 4 - 1] = make_uint4(HD2_UNSET, HD2_UNSET, sub1 | sub2 << 16, sub3);
#pragma unroll
            for (int i = 0; i < (int) (HD2_REFB / 128); ++i)
                bmo[i] = make_uint4(bm[4 * i], bm[4 * i + 1], bm[4 * i + 2], bm[4 * i + 3]);
            if (tab[(size_t) b * HD2_TAB + T_INFO + 2])
            {
                // near-uniform code lengths: no guessing, every entry here (the bitmap in registers)
                for (uint32_t e = 1; e < nent; e += 2)
                {
                    const bool two = e + 1 < nent;
                    uint32_t   ra, rb;
                    hd2_walk_entries(L, payload, payload_off[b], nbytes, s, stop, bm, w0 & ~0xFFFFu, w0 & 0xFFFFu, e, e + 1, two, ra, rb);
                    out[e] = ra;
                    if (two)
                        out[e + 1] = rb;
                }
            }
            continue;
        }
        // HD_GUESS / HD_REST: the entry-0 path's records
        const uint32_t w0 = out[0], c0 = w0 & 0xFFFFu, r0 = w0 & ~0xFFFFu;
        uint32_t       eg = 0;
        if (MODE == HD_GUESS)
        {
            if (tab[(size_t) b * HD2_TAB + T_INFO + 2])
                continue;  // near-uniform code lengths: HD_E0 walked every entry
            if (j == 0)
                continue;
            eg = (trans[(size_t) (g0 + j - 1) * HD2_STRD] >> 16) & 31u;
            if (eg == 0 || eg >= nent)
                continue;  // entry 0: its word is there; >= lmax cannot happen (left unset)
        }
#pragma unroll
        for (int i = 0; i < (int) (HD2_REFB / 128); ++i)
        {
            const uint4 v = bmo[i];
            bm[4 * i] = v.x, bm[4 * i + 1] = v.y, bm[4 * i + 2] = v.z, bm[4 * i + 3] = v.w;
        }
        if (MODE == HD_GUESS)
        {
            uint32_t r, unused;
            hd2_walk_entries(L, payload, payload_off[b], nbytes, s, stop, bm, r0, c0, eg, eg, false, r, unused, true);
            out[eg] = r;
            // (an unjoined word in the block's last segment is the true one all the same: no next
            // segment can be entered off the guess)
            if (r == HD2_UNSET || (!((r >> 30) & 1u) && j + 1 < ns))
            {
                tflag[tk] = 1;  // benign race: every writer stores 1
                if (tk + 1 < ntasks)
                    tflag[tk + 1] = 1;  // its first segment may be entered off the guess
            }
            continue;
        }
        for (uint32_t e = 1; e < nent; e += 2)
        {
            const bool two = e + 1 < nent;
            uint32_t   ra, rb;
            hd2_walk_entries(L, payload, payload_off[b], nbytes, s, stop, bm, r0, c0, e, e + 1, two, ra, rb);
            out[e] = ra;
            if (two)
                out[e + 1] = rb;
        }
    }
}

// Per block: the true path from segment to segment, 256 segments at a time.  Guess: segment k is
// entered where the entry-0 path of segment k - 1 leaves it.  That holds whenever the true path of
// k - 1 joined its entry-0 path (bit 30), so if every guessed word of the chunk but the last has
// bit 30 (the chunk's first segment is entered where the chunk before left), the guesses are the
// true path by induction and the chunk's offsets are one prefix sum -- Huffman codes of unequal
// lengths resynchronise within a few codewords, so text and skewed data take this path.
// Otherwise (codes of near-equal lengths keep separate phases) one lane walks the chunk serially;
// a word it needs that k_hd_trans left unset sets *redo (the host reruns the batch with every
// entry).  Either way the result is the reference's sequential walk: offsets up to orig_size,
// nothing after the first death, fail when the path dies before symbol orig_size.
constexpr uint32_t HD2_CTPB = 256;
__global__ void __launch_bounds__(HD2_CTPB) k_hd_chain(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, const uint32_t* __restrict__ seg_base,
                                                       const uint32_t* __restrict__ trans, uint32_t* __restrict__ seg_info, uint32_t* __restrict__ status,
                                                       uint32_t* __restrict__ redo)
{
    __shared__ uint32_t rows[HD2_CTPB * HD2_STRD];
    __shared__ uint32_t wsum[HD2_CTPB / 64], wdead[HD2_CTPB / 64], sh_e, sh_acc, sh_done, sh_fail, sh_all;
    const uint32_t      t = threadIdx.x, lane = t & 63u, wv = wave_id();
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t g0 = seg_base[b], ns = seg_base[b + 1] - g0, osz = meta[b].orig_size;
        __syncthreads();
        if (t == 0)
        {
            sh_e = 0, sh_acc = 0, sh_done = 0, sh_fail = 0;
        }
        for (uint32_t c0 = 0; c0 < ns; c0 += HD2_CTPB)
        {
            const uint32_t nr = min(HD2_CTPB, ns - c0);
            __syncthreads();
            for (uint32_t i = t; i < nr * HD2_STRD; i += HD2_CTPB)
                rows[i] = trans[(size_t) (g0 + c0) * HD2_STRD + i];
            if (t == 0)
                sh_all = 1;
            __syncthreads();
            const uint32_t e0 = sh_e, acc0 = sh_acc, done0 = sh_done;
            // the guessed entry and word of segment c0 + t
            uint32_t g = 0, word = 0, cnt = 0;
            if (t < nr)
            {
                g    = t == 0 ? e0 : (rows[(t - 1) * HD2_STRD] >> 16) & 31u;
                word = rows[t * HD2_STRD + g];
                cnt  = word & 0xFFFFu;
                // the last word of the chunk need not have joined: the next chunk starts from its
                // exit, carried in sh_e
                if (word == HD2_UNSET || (!((word >> 30) & 1u) && t + 1 < nr))
                    sh_all = 0;  // benign race: every writer stores 0
            }
            // inclusive prefix of the counts and of the death flags over the chunk
            uint32_t inc = cnt, dead = (t < nr) ? (word >> 31) : 0u;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1)
            {
                const uint32_t o = (uint32_t) __shfl_up((int) inc, d, 64), od = (uint32_t) __shfl_up((int) dead, d, 64);
                if ((int) lane >= d)
                    inc += o, dead += od;
            }
            if (lane == 63)
                wsum[wv] = inc, wdead[wv] = dead;
            __syncthreads();
            if (done0)
            {
                if (t < nr)
                    seg_info[g0 + c0 + t] = 0xFFFFFFFFu;  // the path died in an earlier chunk
                continue;
            }
            if (sh_all)
            {
                uint32_t wb = 0, db = 0;
                for (uint32_t i = 0; i < wv; ++i)
                    wb += wsum[i], db += wdead[i];
                inc += wb, dead += db;
                // segment t is walked iff no death strictly before it: deaths up to t minus its own
                const uint32_t before = dead - ((t < nr) ? (word >> 31) : 0u), acc = acc0 + inc - cnt;
                if (t < nr)
                {
                    uint32_t info = 0xFFFFFFFFu;
                    if (before == 0 && acc < osz)
                    {
                        info = (g << 27) | acc;
                        if (word >> 31)
                        {
                            sh_done = 1;  // the one segment with the first death
                            if (acc + cnt < osz)
                                sh_fail = 1;
                        }
                    }
                    seg_info[g0 + c0 + t] = info;
                }
                if (t == nr - 1)
                {
                    sh_acc = acc0 + inc;  // past orig_size or past a death, the sum no longer matters
                    sh_e   = (word >> 16) & 31u;
                }
            }
            else if (t == 0)
            {
                uint32_t e = e0, acc = acc0, done = 0, fail = 0, unset = 0;
                for (uint32_t k = 0; k < nr; ++k)
                {
                    uint32_t info = 0xFFFFFFFFu;
                    if (!done && acc < osz)
                    {
                        const uint32_t r = rows[k * HD2_STRD + e], cnt = r & 0xFFFFu;
                        // a word k_hd_trans left unset (HD_REST skipped the task): the walk goes on
                        // with garbage inside the row and the host reruns the batch with every entry
                        unset |= r == HD2_UNSET ? 1u : 0u;
                        info             = (e << 27) | acc;
                        if (r >> 31)
                        {
                            if (acc + cnt < osz)
                                fail = 1;  // the path dies before symbol orig_size
                            done = 1;
                        }
                        acc += cnt;
                        e = (r >> 16) & 31u;
                    }
                    seg_info[g0 + c0 + k] = info;
                }
                sh_e = e, sh_acc = acc, sh_done = done;
                if (fail)
                    sh_fail = 1;
                if (unset)
                    *redo = 1;
            }
        }
        __syncthreads();
        if (t == 0)
            status[b] = (sh_fail || sh_acc < osz) ? 1u : 0u;
    }
}

// Symbols [0, n) of the path from bit p into dst (a lane writes its own range: 16 bytes per store
// once dst is aligned, dword stores would cost a request per 4 bytes); returns the bit after them.
__device__ __forceinline__ uint32_t hd2_write_run(const Hd2Lds& L, BitWin& W, uint32_t p, uint8_t* dst, uint32_t n)
{
    uint32_t len = 0, sym = 0, i = 0;
    for (; i < n && (((uintptr_t) (dst + i)) & 15); ++i)
    {
        (void) hd2_dec(L, W.peek(p), len, sym);
        p += len;
        dst[i] = (uint8_t) sym;
    }
    for (; i + 16 <= n; i += 16)
    {
        uint32_t wv[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 16; ++k)
        {
            (void) hd2_dec(L, W.peek(p), len, sym);
            p += len;
            wv[k >> 2] |= sym << (8 * (k & 3));
        }
        *reinterpret_cast<uint4*>(dst + i) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
    for (; i < n; ++i)
    {
        (void) hd2_dec(L, W.peek(p), len, sym);
        p += len;
        dst[i] = (uint8_t) sym;
    }
    return p;
}

// Per segment: decode the true path into out[off, off + n), four lanes per segment.  A true path
// that joined the entry-0 path (bit 30 of its transfer word; it joins within the first HD2_REFB
// bits) passes through the entry-0 path's codeword starts recorded after every HD2_SUB bits, so
// lane k > 0 decodes from the k-th record to the next and lane 0 from the entry to the first; a
// path that did not join (codes of near-equal lengths) is decoded by lane 0 alone.  The decode is
// a dependent chain per lane (window bits -> LUT read -> length), so four lanes on a quarter each
// hide its latency four times better.
__global__ void __launch_bounds__(HD2_WTPB) k_hd_write2(const HuffMetaRec* __restrict__ meta, const uint8_t* __restrict__ payload,
                                                        const uint64_t* __restrict__ payload_off, const uint32_t* __restrict__ tab,
                                                        const Hd2Task* __restrict__ tasks, uint32_t ntasks, const uint32_t* __restrict__ seg_base,
                                                        const uint32_t* __restrict__ trans, const uint32_t* __restrict__ seg_info,
                                                        const uint32_t* __restrict__ status, uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_base, uint64_t* __restrict__ end_pos)
{
    __shared__ Hd2Lds L;
    const uint32_t    k = threadIdx.x & 3u;
    for (uint32_t tk = blockIdx.x; tk < ntasks; tk += gridDim.x)
    {
        const Hd2Task  K = tasks[tk];
        const uint32_t b = K.block;
        __syncthreads();
        hd2_load_tables(tab + (size_t) b * HD2_TAB, L);
        const uint32_t j = K.seg0 + (threadIdx.x >> 2), g0 = seg_base[b], ns = seg_base[b + 1] - g0;
        if (j >= ns || status[b])
            continue;
        const uint32_t info = seg_info[g0 + j];
        const uint32_t osz  = meta[b].orig_size;
        if (info == 0xFFFFFFFFu)
            continue;
        const uint32_t e = info >> 27, off = info & 0x7FFFFFFu;
        if (off >= osz)
            continue;
        const uint32_t* tr  = trans + (size_t) (g0 + j) * HD2_STRD;
        const uint32_t  r   = tr[e], cnt = r & 0xFFFFu;
        const uint32_t  n   = min(cnt, osz - off);
        // this lane's symbols [i0, i1) of the segment's cnt, from bit p
        uint32_t i0 = 0, i1 = cnt, p = j * HD2_SEG + e;
        if ((r >> 30) & 1u)
        {
            const uint32_t c0 = tr[0] & 0xFFFFu, s12 = tr[HD2_STRD - 2], s3 = tr[HD2_STRD - 1];
            // records: rank in bits 0-10, offset past the mark above; once one is missing (the
            // path ended before its mark) so are the later ones.  The entry-0 path's codeword of
            // rank x is symbol cnt - c0 + x of the true path.
            const uint32_t mine = k == 1 ? (s12 & 0xFFFFu) : k == 2 ? (s12 >> 16) : s3;
            const uint32_t next = k == 0 ? (s12 & 0xFFFFu) : k == 1 ? (s12 >> 16) : k == 2 ? s3 : 0xFFFFu;
            if (k > 0)
            {
                if (mine == 0xFFFFu)
                    continue;  // the lane before runs to the end
                i0 = cnt - c0 + (mine & 0x7FFu);
                p  = j * HD2_SEG + k * HD2_SUB + (mine >> 11);
            }
            if (next != 0xFFFFu)
                i1 = cnt - c0 + (next & 0x7FFu);
        }
        else if (k > 0)
            continue;
        const uint32_t z = min(i1, n);
        if (i0 >= z)
            continue;
        BitWin W = hd2_win(payload, payload_off[b], meta[b].encoded_size);
        W.init(p);
        p = hd2_write_run(L, W, p, out + out_base[b] + off + i0, z - i0);
        if (off + n == osz && z == n)
            end_pos[b] = p;
    }
}

// Per block: the end-of-stream walk on the intervals.  From the byte boundary after the last symbol
// (bit 0 for orig_size 0) the reference walks the remaining r bits as one codeword: completing a
// symbol or meeting a dead edge within them is an error.  With v = those bits left-justified and
// zero-filled: dead within r bits <=> v >= lim[lmax]; a codeword completes <=> v's interval length
// is <= r (a shorter codeword that is a prefix of the bits would contain v).
__global__ void k_hd_tail2(const HuffMetaRec* __restrict__ meta, uint32_t nblocks, const uint8_t* __restrict__ payload,
                           const uint64_t* __restrict__ payload_off, const uint32_t* __restrict__ tab, const uint64_t* __restrict__ end_pos,
                           uint32_t* __restrict__ status)
{
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += gridDim.x * blockDim.x)
    {
        if (status[b])
            continue;
        const uint32_t  nbytes = meta[b].encoded_size, nbits = nbytes * 8;
        const uint64_t  p2     = meta[b].orig_size ? ((end_pos[b] + 7) & ~7ull) : 0;
        const uint32_t* T      = tab + (size_t) b * HD2_TAB;
        const uint32_t  lmax   = T[T_INFO];
        if (p2 >= nbits)
            continue;
        const uint32_t r = nbits - (uint32_t) p2;
        if (r >= lmax)
        {
            status[b] = 1;  // within lmax bits a walk completes or dies
            continue;
        }
        const uint8_t* src = payload + payload_off[b] + (p2 >> 3);
        uint32_t       v   = 0;
        for (uint32_t k = 0; k < 4; ++k)
            v = (v << 8) | ((p2 >> 3) + k < nbytes ? src[k] : 0u);
        v &= r >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> r);
        const uint64_t* lim = reinterpret_cast<const uint64_t*>(T + T_LIM);
        uint32_t        err = (uint64_t) v >= lim[lmax] ? 1u : 0u;
        if (!err)
            for (uint32_t l = 1; l <= lmax; ++l)
                if ((uint64_t) v < lim[l])
                {
                    err = l <= r ? 1u : 0u;
                    break;
                }
        status[b] = err;
    }
}

}  // namespace

bool HuffWorkspace::reserve(uint32_t nblocks, uint32_t ntiles)
{
    if (nblocks > cap_b)
    {
        cap_b    = 0;
        cap_tree = 0;  // decode buffers allocated lazily (reserve_tree)
        (void) hipFree(tree_child);
        (void) hipFree(tree_sym);
        (void) hipFree(table);
        tree_child = nullptr;
        tree_sym   = nullptr;
        table      = nullptr;
        const uint32_t c = nblocks + 8;
        if (!dev_alloc(codes, (uint64_t) c * 256) || !dev_alloc(status, c))
            return false;
        cap_b = c;
    }
    if (ntiles > cap_t)
    {
        cap_t            = 0;
        const uint32_t c = ntiles + ntiles / 4 + 64;
        if (!dev_alloc(tbits, c) || !dev_alloc(tbit0, c))
            return false;
        cap_t = c;
    }
    return true;
}

bool HuffWorkspace::reserve_tree(uint32_t nblocks)
{
    if (nblocks <= cap_tree)
        return true;
    cap_tree = 0;
    if (!dev_alloc(tree_child, (uint64_t) nblocks * TREE_CAP * 2) || !dev_alloc(tree_sym, (uint64_t) nblocks * TREE_CAP) ||
        !dev_alloc(table, (uint64_t) nblocks * (1u << PEEK)))
        return false;
    cap_tree = nblocks;
    return true;
}

bool HuffWorkspace::reserve_segs(uint32_t nseg, uint32_t nblocks)
{
    if (nseg > cap_seg)
    {
        cap_seg          = 0;
        const uint32_t c = nseg + nseg / 4 + 256;
        if (!dev_alloc_bytes(seg, (uint64_t) c * 3 * sizeof(HdSeg)) || !dev_alloc(seg_off, c))
            return false;
        cap_seg = c;
    }
    if (nblocks + 1 > cap_segb)
    {
        cap_segb         = 0;
        const uint32_t c = nblocks + 64;
        if (!dev_alloc(seg_base, c) || !dev_alloc(end_pos, c) || !dev_alloc(flag, 1))
            return false;
        if (h_flag)
            (void) hipHostFree(h_flag);
        h_flag = nullptr;
        BRA_HIP_CHECK(hipHostMalloc(&h_flag, (size_t) (c + 1) * 4, hipHostMallocDefault));
        cap_segb = c;
    }
    return true;
}

void HuffWorkspace::release()
{
    (void) hipFree(seg);
    (void) hipFree(seg_off);
    (void) hipFree(seg_base);
    (void) hipFree(end_pos);
    (void) hipFree(flag);
    if (h_flag)
        (void) hipHostFree(h_flag);
    tiling.release();
    (void) hipFree(codes);
    (void) hipFree(tbits);
    (void) hipFree(tbit0);
    (void) hipFree(tree_child);
    (void) hipFree(tree_sym);
    (void) hipFree(table);
    (void) hipFree(status);
    (void) hipFree(tab);
    (void) hipFree(trans);
    (void) hipFree(seg_info);
    (void) hipFree(bmbuf);
    (void) hipFree(tflag);
    (void) hipFree(tasks);
    *this = HuffWorkspace{};
}

bool huff_encode_device(HuffWorkspace& w, const uint8_t* d_rle, const BlockDesc* h_rle_cap_blocks, uint32_t nblocks,
                        const uint32_t* d_hist, const uint32_t* d_rle_size, HuffMetaRec* d_meta, uint64_t* d_payload_off,
                        uint8_t* d_payload, uint64_t payload_cap, uint64_t* h_total, hipStream_t s, bool cap_sufficient)
{
    if (!w.tiling.build(h_rle_cap_blocks, nblocks, RLE_TILE, s))
        return false;
    const uint32_t nt = w.tiling.n;
    if (!w.reserve(nblocks, nt))
        return false;
    {
        BRA_PROF(P_HUF_BUILD, s);
        hipLaunchKernelGGL(k_huff_build, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(64), 0, s, d_hist, d_rle_size, nblocks, d_meta, w.codes);
    }
    {
        BRA_PROF(P_HUF_OFFSETS, s);
        hipLaunchKernelGGL(k_huff_offsets, dim3(1), dim3(TPB), 0, s, d_meta, nblocks, d_payload_off);
    }
    const uint32_t grid = std::min<uint32_t>(nt, 32768u);  // workgroups of the tile kernels (8192: 0.03 ms slower per stage)
    {
        BRA_PROF(P_HUF_TILEBITS, s);
        hipLaunchKernelGGL(k_huff_tilebits, dim3(grid), dim3(TPB), 0, s, d_rle, w.tiling.d_pieces, nt, d_meta, w.tbits);
    }
    {
        BRA_PROF(P_HUF_TILESCAN, s);
        hipLaunchKernelGGL(k_huff_tilescan, dim3(std::min<uint32_t>(nblocks, 4096)), dim3(64), 0, s, w.tiling.d_first, w.tiling.d_count, nblocks,
                           d_payload_off, w.tbits, w.tbit0);
    }
    // The payload is at most the RLE bytes plus a word per block (an optimal prefix code over byte
    // symbols is never longer than the 8-bit one): a caller whose capacity covers that bound needs
    // no check, and the stream is not stopped here for it.
    *h_total = 0;
    if (!cap_sufficient)
    {
        BRA_HIP_CHECK(hipMemcpyAsync(h_total, d_payload_off + nblocks, 8, hipMemcpyDeviceToHost, s));
        BRA_HIP_CHECK(hipStreamSynchronize(s));
    }
    if (!cap_sufficient && *h_total + 8 > payload_cap)
    {
        bra_hip_report("huffman: payload capacity %llu too small for %llu bytes", (unsigned long long) payload_cap,
                       (unsigned long long) *h_total);
        return false;
    }
    uint32_t* words = reinterpret_cast<uint32_t*>(d_payload);
    {
        BRA_PROF(P_HUF_ZERO, s);
        hipLaunchKernelGGL(k_huff_zero, dim3(std::min<uint32_t>(div_up(nt, 256), 4096)), dim3(256), 0, s, w.tbits, w.tbit0, nt, words);
    }
    {
        BRA_PROF(P_HUF_PACK, s);
        hipLaunchKernelGGL(k_huff_pack, dim3(xcd_grid(grid)), dim3(TPB), 0, s, d_rle, w.tiling.d_pieces, nt, d_meta, w.codes, w.tbits, w.tbit0, words);
    }
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

// The tree-walking decoder (any code-length set the reference accepts, e.g. codes longer than 30
// bits or an over-full length set the tree rebuild rejects): self-synchronising segments.
static bool huff_decode_tree(HuffWorkspace& w, const HuffMetaRec* d_meta, const uint32_t* h_encoded_size, uint32_t nblocks,
                             const uint8_t* d_payload, const uint64_t* d_payload_off, uint8_t* d_out, const uint64_t* d_out_base,
                             uint32_t* d_status, hipStream_t s)
{
    if (!w.reserve(nblocks, 1) || !w.reserve_tree(nblocks))
        return false;
    hipLaunchKernelGGL(k_huff_tree, dim3(div_up(nblocks, 64)), dim3(64), 0, s, d_meta, nblocks, w.tree_child, w.tree_sym, w.status);
    hipLaunchKernelGGL(k_huff_table, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(256), 0, s, w.tree_child, w.tree_sym, nblocks, w.table);
    // segments per block from the host-side encoded sizes
    if (!w.reserve_segs(1, nblocks))
        return false;
    uint32_t* hb = w.h_flag + 1;  // pinned: segment bases, then one more entry for the total
    uint32_t  ns = 0;
    for (uint32_t b = 0; b < nblocks; ++b)
    {
        hb[b] = ns;
        ns += (uint32_t) div_up((uint64_t) h_encoded_size[b] * 8, SEG_BITS);
    }
    hb[nblocks] = ns;
    if (!w.reserve_segs(ns, nblocks))
        return false;
    hb = w.h_flag + 1;  // (reserve may have reallocated the pinned buffer before the copy below)
    {
        uint32_t n2 = 0;
        for (uint32_t b = 0; b < nblocks; ++b)
        {
            hb[b] = n2;
            n2 += (uint32_t) div_up((uint64_t) h_encoded_size[b] * 8, SEG_BITS);
        }
        hb[nblocks] = n2;
    }
    BRA_HIP_CHECK(hipMemcpyAsync(w.seg_base, hb, (size_t) (nblocks + 1) * 4, hipMemcpyHostToDevice, s));
    HdSeg* spec = reinterpret_cast<HdSeg*>(w.seg);
    HdSeg* cur  = spec + w.cap_seg;
    HdSeg* nxt  = cur + w.cap_seg;
    const uint32_t grid = std::min<uint32_t>(div_up(std::max(ns, 1u), 256), 16384);
    if (ns)
    {
        hipLaunchKernelGGL(k_hd_spec, dim3(grid), dim3(256), 0, s, d_meta, nblocks, d_payload, d_payload_off, w.tree_child, w.tree_sym, w.table,
                           w.status, w.seg_base, ns, spec);
        BRA_HIP_CHECK(hipMemcpyAsync(cur, spec, (size_t) ns * sizeof(HdSeg), hipMemcpyDeviceToDevice, s));
        for (int it = 0; it < 64; ++it)
        {
            BRA_HIP_CHECK(hipMemsetAsync(w.flag, 0, 4, s));
            hipLaunchKernelGGL(k_hd_sync, dim3(grid), dim3(256), 0, s, d_meta, nblocks, d_payload, d_payload_off, w.tree_child, w.tree_sym,
                               w.table, w.status, w.seg_base, ns, spec, cur, nxt, w.flag);
            BRA_HIP_CHECK(hipMemcpyAsync(w.h_flag, w.flag, 4, hipMemcpyDeviceToHost, s));
            BRA_HIP_CHECK(hipStreamSynchronize(s));
            std::swap(cur, nxt);
            if (!*w.h_flag)
                break;
        }
    }
    hipLaunchKernelGGL(k_hd_prefix, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(256), 0, s, d_meta, nblocks, w.status, w.seg_base, cur,
                       w.seg_off, d_status);
    if (ns)
        hipLaunchKernelGGL(k_hd_write, dim3(grid), dim3(256), 0, s, d_meta, nblocks, d_payload, d_payload_off, w.tree_child, w.tree_sym, w.table,
                           d_status, w.seg_base, ns, cur, w.seg_off, d_out, d_out_base, w.end_pos);
    hipLaunchKernelGGL(k_hd_tail, dim3(div_up(nblocks, 64)), dim3(64), 0, s, d_meta, nblocks, d_payload, d_payload_off, w.tree_child, w.tree_sym,
                       w.table, w.end_pos, d_status);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

// Test hook (tests/test_gpu_parity.py): BRA_HD_TEST_UNMARK=1 clears the task marks of the
// guessing pass, so every true path that leaves the guesses meets unset words in the chain and the
// batch takes the rerun with every entry.  Read per call.
static bool hd_test_unmark()
{
    const char* e = getenv("BRA_HD_TEST_UNMARK");
    return e && e[0] == '1';
}

bool huff_decode_device(HuffWorkspace& w, const HuffMetaRec* d_meta, const uint32_t* h_encoded_size, uint32_t nblocks, const uint8_t* d_payload,
                        const uint64_t* d_payload_off, uint8_t* d_out, const uint64_t* d_out_base, uint32_t* d_status, hipStream_t s)
{
    if (nblocks == 0)
        return true;
    if (!w.reserve(nblocks, 1) || !w.reserve_segs(1, nblocks))
        return false;
    // segments and WG tasks from the host-side encoded sizes
    std::vector<uint32_t>& hb = w.h_segb;
    hb.resize(nblocks + 1);
    std::vector<Hd2Task> tasks;
    tasks.reserve(nblocks);
    uint32_t ns = 0;
    for (uint32_t b = 0; b < nblocks; ++b)
    {
        hb[b]            = ns;
        const uint32_t n = (uint32_t) div_up((uint64_t) h_encoded_size[b] * 8, HD2_SEG);
        for (uint32_t j = 0; j < n; j += HD2_TPB)
            tasks.push_back(Hd2Task{b, j});
        ns += n;
    }
    hb[nblocks] = ns;
    const uint32_t nt = (uint32_t) tasks.size();
    if (!w.reserve_fast(nblocks, ns, nt))
        return false;
    BRA_HIP_CHECK(hipMemsetAsync(w.flag, 0, 4, s));
    BRA_HIP_CHECK(hipMemcpyAsync(w.seg_base, hb.data(), (size_t) (nblocks + 1) * 4, hipMemcpyHostToDevice, s));
    if (nt)
        BRA_HIP_CHECK(hipMemcpyAsync(w.tasks, tasks.data(), (size_t) nt * sizeof(Hd2Task), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_hd_canon, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(256), 0, s, d_meta, nblocks, w.tab, w.flag);
    BRA_HIP_CHECK(hipMemcpyAsync(w.h_flag, w.flag, 4, hipMemcpyDeviceToHost, s));
    BRA_HIP_CHECK(hipStreamSynchronize(s));  // also: the host vectors above were the copies' sources
    if (*w.h_flag)
        return huff_decode_tree(w, d_meta, h_encoded_size, nblocks, d_payload, d_payload_off, d_out, d_out_base, d_status, s);
    const Hd2Task* dt = reinterpret_cast<const Hd2Task*>(w.tasks);
    if (nt)
    {
        BRA_PROF(P_DEC_HD_TRANS, s);
        if (g_prof)
        {
            double hb = 0;  // algorithmic bytes: the payload, read once
            for (uint32_t b = 0; b < nblocks; ++b)
                hb += h_encoded_size[b];
            prof_bytes(P_DEC_HD_TRANS, hb);
        }
        const dim3 g(std::min<uint32_t>(nt, 65535));
        BRA_HIP_CHECK(hipMemsetAsync(w.tflag, 0, (size_t) (nt + 1) * 4, s));
        hipLaunchKernelGGL(k_hd_trans<HD_E0>, g, dim3(HD2_TPB), 0, s, d_meta, d_payload, d_payload_off, w.tab, dt, nt, w.seg_base, w.trans, w.bmbuf,
                           w.tflag);
        hipLaunchKernelGGL(k_hd_trans<HD_GUESS>, g, dim3(HD2_TPB), 0, s, d_meta, d_payload, d_payload_off, w.tab, dt, nt, w.seg_base, w.trans,
                           w.bmbuf, w.tflag);
        if (hd_test_unmark())
            BRA_HIP_CHECK(hipMemsetAsync(w.tflag, 0, (size_t) nt * 4, s));
        hipLaunchKernelGGL(k_hd_trans<HD_REST>, g, dim3(HD2_TPB), 0, s, d_meta, d_payload, d_payload_off, w.tab, dt, nt, w.seg_base, w.trans,
                           w.bmbuf, w.tflag);
    }
    hipLaunchKernelGGL(k_hd_chain, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(HD2_CTPB), 0, s, d_meta, nblocks, w.seg_base, w.trans, w.seg_info,
                       d_status, nt ? w.tflag + nt : w.flag);  // no task: no segment, the flag is never written
    *w.h_flag = 0;
    if (nt)
    {
        BRA_HIP_CHECK(hipMemcpyAsync(w.h_flag, w.tflag + nt, 4, hipMemcpyDeviceToHost, s));
        BRA_HIP_CHECK(hipStreamSynchronize(s));
    }
    if (*w.h_flag)
    {
        // a true path left the guessed entries where HD_REST had not run: every entry, then the chain again
        BRA_HIP_CHECK(hipMemsetAsync(w.tflag, 1, (size_t) nt * 4, s));
        BRA_HIP_CHECK(hipMemsetAsync(w.tflag + nt, 0, 4, s));
        hipLaunchKernelGGL(k_hd_trans<HD_REST>, dim3(std::min<uint32_t>(nt, 65535)), dim3(HD2_TPB), 0, s, d_meta, d_payload, d_payload_off, w.tab,
                           dt, nt, w.seg_base, w.trans, w.bmbuf, w.tflag);
        hipLaunchKernelGGL(k_hd_chain, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(HD2_CTPB), 0, s, d_meta, nblocks, w.seg_base, w.trans,
                           w.seg_info, d_status, w.tflag + nt);
    }
    if (nt)
        hipLaunchKernelGGL(k_hd_write2, dim3(std::min<uint32_t>(nt, 65535)), dim3(HD2_WTPB), 0, s, d_meta, d_payload, d_payload_off, w.tab, dt, nt,
                           w.seg_base, w.trans, w.seg_info, d_status, d_out, d_out_base, w.end_pos);
    hipLaunchKernelGGL(k_hd_tail2, dim3(div_up(nblocks, 64)), dim3(64), 0, s, d_meta, nblocks, d_payload, d_payload_off, w.tab, w.end_pos,
                       d_status);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

bool HuffWorkspace::reserve_fast(uint32_t nblocks, uint32_t nseg, uint32_t ntasks)
{
    if (nblocks > cap_fb)
    {
        cap_fb           = 0;
        const uint32_t c = nblocks + 64;
        if (!dev_alloc(tab, (uint64_t) c * HD2_TAB))
            return false;
        cap_fb = c;
    }
    if (nseg > cap_fs)
    {
        cap_fs           = 0;
        const uint32_t c = nseg + nseg / 4 + 256;
        if (!dev_alloc(trans, (uint64_t) c * HD2_STRD) || !dev_alloc(seg_info, c) || !dev_alloc(bmbuf, (uint64_t) c * (HD2_REFB / 32)))
            return false;
        cap_fs = c;
    }
    if (ntasks > cap_ft)
    {
        cap_ft           = 0;
        const uint32_t c = ntasks + ntasks / 4 + 64;
        if (!dev_alloc_bytes(tasks, (uint64_t) c * sizeof(Hd2Task)) || !dev_alloc(tflag, (uint64_t) c + 1))
            return false;
        cap_ft = c;
    }
    return true;
}

namespace {
__global__ void __launch_bounds__(256) k_hist256(const uint8_t* __restrict__ in, const Piece* __restrict__ tiles, uint32_t ntiles,
                                                 uint32_t* __restrict__ hist)
{
    __shared__ uint32_t h[256];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        h[threadIdx.x] = 0;
        __syncthreads();
        const Piece P = tiles[t];
        for (uint32_t i = threadIdx.x; i < P.len; i += 256)
            atomicAdd(&h[in[P.off + i]], 1u);
        __syncthreads();
        if (h[threadIdx.x])
            atomicAdd(&hist[(size_t) P.block * 256 + threadIdx.x], h[threadIdx.x]);
        __syncthreads();
    }
}
}  // namespace

bool histogram_device(Tiling& tiling, const uint8_t* d_in, const BlockDesc* h_blocks, uint32_t nblocks, uint32_t* d_hist, hipStream_t s)
{
    if (!tiling.build(h_blocks, nblocks, RLE_TILE, s))
        return false;
    BRA_HIP_CHECK(hipMemsetAsync(d_hist, 0, (size_t) nblocks * 256 * 4, s));
    if (tiling.n)
        hipLaunchKernelGGL(k_hist256, dim3(std::min<uint32_t>(tiling.n, 8192)), dim3(256), 0, s, d_in, tiling.d_pieces, tiling.n, d_hist);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace bra
