// mtf.hip -- move-to-front encode/decode for a batch of independent blocks.
//
// Replaces bra_mtf_encode2 / bra_mtf_decode2 (reference src/encoders/bra_mtf.c:67-82, :98-115;
// table init :9-13, encode step :16-32 = output position then move to front, decode step :35-46).
//
// Encode is made segment-parallel with the recency formulation: the MTF table at any point lists
// symbols by decreasing last-occurrence time, never-seen symbols last in ascending order (the
// initial identity table is the recency order of a virtual prefix 255, 254, ..., 0).  So
//   k_mtf_presence / k_mtf_alpha   each block's alphabet (from the BWT's presence masks when the
//                      caller has them): distinct symbols, alphabet index of every value, and the
//                      block's encoder: position tables (<= 32 values, all below 127: text, small
//                      alphabets), register byte tables (other <= 32-symbol blocks) or waves;
//   k_mtf_lastocc   last occurrence of every symbol inside each segment (LDS atomicMax); for a
//                   position-table block, of its <= 32 alphabet values inside each HALF segment;
//   k_mtf_scan      exclusive max-scan over the (half) segments of a block -> start-of-segment
//                   times; position-table blocks: the start position table of every half segment;
//   k_mtf_encode_pos   position-table blocks: one thread per 512-byte half segment;
//   k_mtf_encode_reg   other blocks of <= MTF_REG distinct symbols: one thread per segment, the
//                      table front in registers;
//   k_mtf_encode_wave  larger alphabets: one wave per segment, 64 symbols per step (ballots).
// Decode uses relabelling: a decode step moves table POSITION p to the front whatever the table
// holds, so decoding a segment from the identity table gives labels u_i and an end permutation
// P_k; the true start tables satisfy S_{k+1}[j] = S_k[P_k[j]] and the output is S_k[u_i].
#include "mtf.h"
#include "prof.h"

namespace bra {

namespace {

constexpr int TPB = 256;

__device__ __forceinline__ uint32_t haszero8(uint32_t x) { return (x - 0x01010101u) & ~x & 0x80808080u; }

// ------------------------------------------------------------------------------------------------
// encode
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_barrier_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Presence masks when the caller has none: one wave per segment ORs its bytes into 8 mask dwords
// and adds them to its block's mask (amask zeroed by the caller).
__global__ void __launch_bounds__(TPB) k_mtf_presence(const uint8_t* __restrict__ in, const Piece* __restrict__ segs, uint32_t nseg,
                                                      uint32_t* __restrict__ amask)
{
    const int      lane = lane_id();
    const uint32_t wave = wave_id();
    for (uint32_t s = blockIdx.x * (TPB / 64) + wave; s < nseg; s += gridDim.x * (TPB / 64))
    {
        const Piece P = segs[s];
        uint32_t    m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t i = lane; i < P.len; i += 64)
        {
            const uint32_t v = in[P.off + i];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                m[k] |= ((v >> 5) == (uint32_t) k) ? (1u << (v & 31)) : 0u;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
        {
            const uint32_t x = wave_scan<true>(m[k], 0u, OpOr());
            if (lane == 63 && x)
                atomicOr(&amask[8 * (size_t) P.block + k], x);
        }
    }
}

// One workgroup per block, thread c = byte value c: the block's alphabet from its presence mask.
// amap[b][c] = rank of c among the present values (0xFF: absent), ainv[b][a] = the a-th present
// value (a < 32), amode[b] = the position-table dwords (4 for at most 16 values, else ceil(values / 4) up to 32
// distinct values, all below 127 (every MTF position then stays below 127), else 0.
__global__ void __launch_bounds__(TPB) k_mtf_alpha(const uint32_t* __restrict__ amask, uint32_t nblocks, uint32_t* __restrict__ nsym,
                                                   uint8_t* __restrict__ amap, uint8_t* __restrict__ ainv, uint32_t* __restrict__ amode)
{
    __shared__ uint32_t tmp[8];
    const uint32_t      c = threadIdx.x;
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const bool     pres = (amask[8 * (size_t) b + (c >> 5)] >> (c & 31)) & 1u;
        const int      n    = __syncthreads_count(pres);
        const bool     high = __syncthreads_or(pres && c >= 127) != 0;
        const uint32_t rk   = block256_exclusive_sum(pres ? 1u : 0u, tmp);
        amap[(size_t) b * 256 + c] = pres ? (uint8_t) rk : (uint8_t) 0xFF;
        if (pres && rk < 32)
            ainv[(size_t) b * 32 + rk] = (uint8_t) c;
        if (c == 0)
        {
            nsym[b]  = (uint32_t) n;
            amode[b] = (high || n > 32) ? 0u : (n <= 16 ? 4u : (uint32_t) (n + 3) / 4);  // table dwords (4..8)
        }
        __syncthreads();
    }
}

// One wave per segment (1024 symbols = 16 per lane, one 16-byte load): each lane keeps only the
// last byte of every run of equal bytes inside its 16 and max-updates the segment's 256 LDS
// entries; the state row goes out as one 16-byte store per lane.  (A workgroup per segment with a
// 4-byte load per thread was bound by its load -> atomics -> barrier -> store latency chain.)
// Position-table blocks: the lanes of each half segment (lanes 0-31: bytes 0-511) update their own
// row, and the segment's state is two compact rows, [256 s + 32 h + a] = last occurrence of the
// block's a-th value in half h (-1: none; a >= the block's alphabet: -1).  Their values are below
// 127 and few, so many lanes of one atomic instruction hit the same entry (same-address atomics
// serialise: half the kernel's time on text): each half keeps LO_NC copies of its row (copy = lane
// mod LO_NC, LO_CS words apart so one value's copies sit in different banks), merged at the end.
constexpr int LO_NC = 4, LO_CS = 132;
__global__ void __launch_bounds__(TPB) k_mtf_lastocc(const uint8_t* __restrict__ in, const Piece* __restrict__ segs, uint32_t nseg,
                                                     int32_t* __restrict__ state, const uint32_t* __restrict__ amode,
                                                     const uint32_t* __restrict__ nsym, const uint8_t* __restrict__ ainv)
{
    constexpr int      ROW = 2 * LO_NC * LO_CS;  // >= 256: the full row of other blocks
    __shared__ __attribute__((aligned(16))) int32_t lo_s[TPB / 64][ROW];
    const int          lane = lane_id();
    const uint32_t     wave = wave_id();
    for (uint32_t s = blockIdx.x * (TPB / 64) + wave; s < nseg; s += gridDim.x * (TPB / 64))
    {
        const Piece    P    = segs[s];
        const bool     half = amode[P.block] != 0;
        int32_t*       lo   = half ? lo_s[wave] + ((lane >> 5) * LO_NC + (lane & (LO_NC - 1))) * LO_CS : lo_s[wave];
        if (half)
            for (int i = lane; i < ROW / 4; i += 64)
                reinterpret_cast<int4*>(lo_s[wave])[i] = make_int4(-1, -1, -1, -1);
        else
            reinterpret_cast<int4*>(lo_s[wave])[lane] = make_int4(-1, -1, -1, -1);
        const uint8_t* p    = in + P.off;
        const uint32_t i0   = (uint32_t) lane * 16;
        uint32_t       w[4] = {0, 0, 0, 0};
        const uint32_t n    = P.len > i0 ? min(16u, P.len - i0) : 0u;
        if (n == 16 && (((uintptr_t) (p + i0)) & 15) == 0)
        {
            const uint4 v = *reinterpret_cast<const uint4*>(p + i0);
            w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
        }
        else
            for (uint32_t j = 0; j < n; ++j)
                w[j >> 2] |= (uint32_t) p[i0 + j] << (8 * (j & 3));
        wave_barrier_lds();
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j)
        {
            const uint32_t c  = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t cn = (w[(j + 1) >> 2 & 3] >> (8 * ((j + 1) & 3))) & 0xFFu;
            if (j < n && (j + 1 == n || c != cn))
                atomicMax(&lo[c], (int32_t) (i0 + j));
        }
        wave_barrier_lds();
        const int32_t st = (int32_t) P.start;
        if (half)
        {
            const uint32_t a = (uint32_t) lane & 31u;
            int32_t        v = -1;
            if (a < nsym[P.block])
            {
                const int32_t* row = lo_s[wave] + (lane >> 5) * LO_NC * LO_CS + ainv[(size_t) P.block * 32 + a];
#pragma unroll
                for (int k = 0; k < LO_NC; ++k)
                    v = max(v, row[k * LO_CS]);
            }
            state[(size_t) s * 256 + lane] = v >= 0 ? st + v : -1;
        }
        else
        {
            const int4 v = reinterpret_cast<const int4*>(lo)[lane];
            reinterpret_cast<int4*>(state + (size_t) s * 256)[lane] =
                make_int4(v.x >= 0 ? st + v.x : -1, v.y >= 0 ? st + v.y : -1, v.z >= 0 ? st + v.z : -1, v.w >= 0 ? st + v.w : -1);
        }
        wave_barrier_lds();
    }
}

// ---- position-table blocks: start tables of the half segments, in three parallel passes ----
// Half segment h of segment s: state ints [256 s + 32 (h & 1), +32) hold its last occurrences (one
// per alphabet index a); chunks of PT_CHUNK consecutive half segments of a block, one half wave
// (lane a) per chunk.
constexpr uint32_t PT_CHUNK = 32;

struct PtGeo
{
    const uint32_t* first_seg;   // per block: first segment
    const uint32_t* nseg_blk;    // per block: segments
    const uint32_t* chunk0;      // per block: first chunk (exclusive prefix of ceil(2 ns / PT_CHUNK))
    const uint32_t* chunk_blk;   // per chunk: block
    uint32_t        nchunks;
};

__device__ __forceinline__ int32_t* pt_row(int32_t* state, uint32_t s0, uint32_t h, uint32_t a)
{
    return state + (size_t) (s0 + (h >> 1)) * 256 + (h & 1) * 32 + a;
}

// Pass 1: the maximum of every chunk (cmax[32 c + a]).
__global__ void __launch_bounds__(TPB) k_mtf_pt_max(int32_t* __restrict__ state, PtGeo g, const uint32_t* __restrict__ amode, int32_t* __restrict__ cmax)
{
    const uint32_t a = threadIdx.x & 31u;
    for (uint32_t c = blockIdx.x * (TPB / 32) + (threadIdx.x >> 5); c < g.nchunks; c += gridDim.x * (TPB / 32))
    {
        const uint32_t b = g.chunk_blk[c];
        if (!amode[b])
            continue;
        const uint32_t s0 = g.first_seg[b], H = 2 * g.nseg_blk[b], h0 = (c - g.chunk0[b]) * PT_CHUNK, h1 = min(H, h0 + PT_CHUNK);
        int32_t        v[PT_CHUNK];
#pragma unroll
        for (uint32_t u = 0; u < PT_CHUNK; ++u)
            v[u] = h0 + u < h1 ? *pt_row(state, s0, h0 + u, a) : -1;
        int32_t m = -1;
#pragma unroll
        for (uint32_t u = 0; u < PT_CHUNK; ++u)
            m = max(m, v[u]);
        cmax[32 * (size_t) c + a] = m;
    }
}

// Pass 2, one workgroup per block: exclusive max-scan of its chunk maxima, in place (8 groups of 32
// threads over consecutive eighths, group maxima through LDS).
__global__ void __launch_bounds__(TPB) k_mtf_pt_scan(PtGeo g, uint32_t nblocks, const uint32_t* __restrict__ amode, int32_t* __restrict__ cmax)
{
    __shared__ int32_t agg[8][32];
    const uint32_t     a = threadIdx.x & 31u, gr = threadIdx.x >> 5;
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        if (!amode[b])
            continue;
        const uint32_t c0 = g.chunk0[b], nc = div_up(2ull * g.nseg_blk[b], PT_CHUNK), C = div_up(nc, 8u);
        const uint32_t k0 = min(nc, gr * C), k1 = min(nc, k0 + C);
        int32_t        m = -1;
        for (uint32_t k = k0; k < k1; ++k)
            m = max(m, cmax[32 * (size_t) (c0 + k) + a]);
        agg[gr][a] = m;
        __syncthreads();
        int32_t run = -1;
        for (uint32_t q = 0; q < gr; ++q)
            run = max(run, agg[q][a]);
        for (uint32_t k = k0; k < k1; ++k)
        {
            int32_t* p = cmax + 32 * (size_t) (c0 + k) + a;
            const int32_t v = *p;
            *p              = run;
            run             = max(run, v);
        }
        __syncthreads();  // agg is rewritten by the next block
    }
}

// Pass 3: every half segment's start position table from its chunk's prefix: byte a of the 32 bytes
// at state byte 1024 s + 512 + 32 (h & 1) = 0x80 | the position of the block's a-th value (seen
// values: the number of values seen later; unseen ones follow the seen ones by value), 0xFF beyond
// the alphabet -- the table k_mtf_encode_pos starts from.
__global__ void __launch_bounds__(TPB) k_mtf_pt_tables(int32_t* __restrict__ state, PtGeo g, const uint32_t* __restrict__ amode,
                                                       const uint32_t* __restrict__ nsym, const uint8_t* __restrict__ ainv,
                                                       const int32_t* __restrict__ cpre)
{
    const uint32_t a = threadIdx.x & 31u, hb = (uint32_t) lane_id() & 32u;
    uint8_t*       pt = reinterpret_cast<uint8_t*>(state);
    __shared__ __attribute__((aligned(16))) int32_t tt_s[TPB / 32][32];  // per half wave: the 32 last occurrences
    int32_t*       tts = tt_s[threadIdx.x >> 5];
    for (uint32_t c = blockIdx.x * (TPB / 32) + (threadIdx.x >> 5); c < g.nchunks; c += gridDim.x * (TPB / 32))
    {
        const uint32_t b = g.chunk_blk[c];  // uniform per half wave
        if (!amode[b])
            continue;
        const uint32_t s0 = g.first_seg[b], H = 2 * g.nseg_blk[b], h0 = (c - g.chunk0[b]) * PT_CHUNK, h1 = min(H, h0 + PT_CHUNK);
        const uint32_t na = nsym[b], val = a < na ? ainv[(size_t) b * 32 + a] : 0u;
        int32_t        run = cpre[32 * (size_t) c + a];
        int32_t        v[PT_CHUNK];
#pragma unroll
        for (uint32_t u = 0; u < PT_CHUNK; ++u)
            v[u] = h0 + u < h1 ? *pt_row(state, s0, h0 + u, a) : -1;
        for (uint32_t h = h0; h < h1; ++h)
        {
            int32_t nv = v[0];
#pragma unroll
            for (uint32_t u = 0; u + 1 < PT_CHUNK; ++u)  // shift the chunk's rows down by one (constant indices)
                v[u] = v[u + 1];
            const int32_t  tt   = run;  // last occurrence before half segment h
            run                 = max(run, nv);
            const bool     seen = a < na && tt >= 0;
            const uint32_t mk   = (uint32_t) (__builtin_amdgcn_ballot_w64(seen) >> hb);
            uint32_t       later = 0;
            // the half wave's 32 values through LDS, 4 per broadcast read (32 lane permutes per
            // half segment bounded the kernel)
            tts[a] = tt;
            wave_barrier_lds();
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j)
            {
                const int4 q = reinterpret_cast<const int4*>(tts)[j];
                later += (q.x > tt ? 1u : 0u) + (q.y > tt ? 1u : 0u) + (q.z > tt ? 1u : 0u) + (q.w > tt ? 1u : 0u);
            }
            wave_barrier_lds();
            const uint32_t pos = seen ? later : (uint32_t) __popc(mk) + val - (uint32_t) __popc(mk & ((1u << a) - 1u));
            pt[(size_t) (s0 + (h >> 1)) * 1024 + 512 + (h & 1) * 32 + a] = a < na ? (uint8_t) (0x80u | pos) : (uint8_t) 0xFF;
        }
    }
}

// One workgroup per block; thread c scans symbol c over the block's segments (exclusive max);
// position-table blocks are the k_mtf_pt_* passes'.
__global__ void __launch_bounds__(TPB) k_mtf_scan(const uint32_t* __restrict__ first_seg, const uint32_t* __restrict__ nseg_blk,
                                                  uint32_t nblocks, int32_t* __restrict__ state, const uint32_t* __restrict__ nsym,
                                                  const uint8_t* __restrict__ ainv, const uint32_t* __restrict__ amode)
{
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t s0  = first_seg[b];
        const uint32_t ns  = nseg_blk[b];
        if (amode[b])
            continue;  // k_mtf_pt_*
        int32_t        run = -1;
        const uint32_t c   = threadIdx.x;
        uint32_t       k   = 0;
        // 32 segment rows in flight per round (the scan is a chain of load latencies: 8 per round
        // took 0.13 ms per batch)
        for (; k + 32 <= ns; k += 32)
        {
            int32_t v[32];
#pragma unroll
            for (int u = 0; u < 32; ++u)
                v[u] = state[(size_t) (s0 + k + u) * 256 + c];
#pragma unroll
            for (int u = 0; u < 32; ++u)
            {
                state[(size_t) (s0 + k + u) * 256 + c] = run;
                run                                    = max(run, v[u]);
            }
        }
        for (; k < ns; ++k)
        {
            const int32_t v                       = state[(size_t) (s0 + k) * 256 + c];
            state[(size_t) (s0 + k) * 256 + c] = run;
            run                                   = max(run, v);
        }
    }
}

// Stage (SIZE, J) of a bitonic network over 256 unique 32-bit keys, 4 per lane (slot 4 lane + r),
// ascending, and recursively the rest of its merge phase: partners J >= 4 slots away sit J / 4
// lanes away (DPP / permlane, xlane), closer ones in the same lane.  A compare-exchange of 32-bit
// keys is a min, a max and a select.
template <int SIZE, int J>
__device__ __forceinline__ void sort256_stage(uint32_t (&k)[4])
{
    const uint32_t e0 = (uint32_t) lane_id() * 4;
    if constexpr (J >= 4)
    {
        const bool keep_min = ((e0 & SIZE) == 0) == ((e0 & J) == 0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t o = xlane<J / 4>(k[r]);
            k[r]             = keep_min ? min(k[r], o) : max(k[r], o);
        }
    }
    else
    {
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const int q = r ^ J;
            if (q > r)
            {
                const bool     asc = ((e0 + r) & SIZE) == 0;
                const uint32_t lo = min(k[r], k[q]), hi = max(k[r], k[q]);
                k[r]              = asc ? lo : hi;
                k[q]              = asc ? hi : lo;
            }
        }
    }
    if constexpr (J > 1)
        sort256_stage<SIZE, J / 2>(k);
}

template <int SIZE>
__device__ __forceinline__ void sort256_phases(uint32_t (&k)[4])
{
    sort256_stage<SIZE, SIZE / 2>(k);
    if constexpr (SIZE < 256)
        sort256_phases<SIZE * 2>(k);
}

// Lane l's dword of a segment's start table (entries 4l .. 4l+3, little-endian): the symbols by
// decreasing last occurrence, then the unseen ones by increasing value.  32-bit sort keys: seen
// symbol c: (0xFFFFFE - last occurrence) << 8 | c (occurrences are block positions < 2^24 - 2; larger
// ones take a two-pass form below),
// unseen: 0xFFFFFF00 | c.  (A generic 64-bit key/value sort with LDS permutes here cost about a
// third of the wave kernel's time on uniform random data.)
__device__ __forceinline__ uint32_t start_table_dword(const int32_t* __restrict__ st)
{
    const int  lane = lane_id();
    const int4 tv   = reinterpret_cast<const int4*>(st)[lane];
    const int32_t tt[4] = {tv.x, tv.y, tv.z, tv.w};
    uint32_t   k[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        const uint32_t c = (uint32_t) lane * 4 + r;
        k[r]             = tt[r] >= 0 ? ((0xFFFFFEu - (uint32_t) tt[r]) << 8) | c : 0xFFFFFF00u | c;
    }
    if (__builtin_expect(__any(tv.x >= 0xFFFFFE || tv.y >= 0xFFFFFE || tv.z >= 0xFFFFFE || tv.w >= 0xFFFFFE), 0))
    {
        // a position past 24 bits (single-block C-ABI buffers of 2^24 bytes or more): order by
        // D = 2^31 - 1 - last occurrence (unseen: 2^32 - 1), then c, as two passes over 24-bit
        // digits -- the low 24 bits of D first, then its high 8 bits with the first pass's rank as
        // the tie-break (bitonic sorts are not stable; the rank makes the second pass exact)
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c = (uint32_t) lane * 4 + r;
            const uint32_t D = tt[r] >= 0 ? 0x7FFFFFFFu - (uint32_t) tt[r] : 0xFFFFFFFFu;
            k[r]             = (D & 0xFFFFFFu) << 8 | c;
        }
        sort256_phases<2>(k);
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c  = k[r] & 0xFFu;
            const int32_t  tc = st[c];
            const uint32_t D  = tc >= 0 ? 0x7FFFFFFFu - (uint32_t) tc : 0xFFFFFFFFu;
            k[r]              = (D >> 24) << 16 | ((uint32_t) lane * 4 + r) << 8 | c;
        }
    }
    sort256_phases<2>(k);
    return (k[0] & 0xFF) | ((k[1] & 0xFF) << 8) | ((k[2] & 0xFF) << 16) | ((k[3] & 0xFF) << 24);
}

// Shift one table dword up by one entry: entry 0 becomes the top entry of the previous dword.
__device__ __forceinline__ uint32_t shift1(uint32_t cur, uint32_t below_top) { return (cur << 8) | below_top; }

// Partial shift of the dword holding the symbol at byte b: entries [0, b] move up by one (the
// symbol's own slot is overwritten), entries above b stay.
__device__ __forceinline__ uint32_t shift_upto(uint32_t cur, uint32_t below_top, uint32_t b)
{
    const uint32_t keep = (b == 3) ? 0u : (0xFFFFFFFFu << (8 * (b + 1)));
    return (cur & keep) | (((cur << 8) | below_top) & ~keep);
}

// ---- register tables: blocks of at most MTF_REG distinct symbols ----
// Once a symbol has occurred it stays among the first (distinct symbols) positions of the table, so
// with <= 32 distinct symbols per block the first 32 entries (8 dwords in registers) hold every
// symbol that can be found by a search; entries beyond are byte values not yet seen in the block,
// in increasing value order (true of the identity start table and kept by every move-to-front,
// since the entry pushed out of the register part is then always an unseen value smaller than every
// unseen value behind it).  A symbol not in registers therefore has rank
// MTF_REG + #(unseen values below it) = MTF_REG + c - #(register entries below c).  No LDS table:
// occupancy is bounded by registers, not by a 272-byte LDS row per thread.
constexpr int NRD = MTF_REG / 4;  // register dwords

__device__ __noinline__ uint32_t count_below(const uint32_t (&R)[NRD], uint32_t c)
{
    uint32_t n = 0;
#pragma unroll
    for (int k = 0; k < NRD; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            n += ((R[k] >> (8 * j)) & 0xFFu) < c ? 1u : 0u;
    return n;
}

// One MTF step on the 32-entry register table: the symbol's position p = 4 k + b from the first
// register holding a zero byte of R ^ c (k = 8: not among the first 32 entries -- a first
// occurrence), then every register below k shifts up by one byte (v_alignbit) and register k
// shifts its bytes 0..b (a bitfield insert), all branch-free.  Post-BWT text rarely has all 64
// lanes of a wave inside the first 16 entries at once (P(rank < 16)^64), so a fast path for them
// rarely ran and the per-register branches cost more than they saved.
__device__ __forceinline__ uint32_t mtf_step_reg(uint32_t (&R)[NRD], uint32_t c)
{
    const uint32_t cc = c * 0x01010101u;
    uint32_t       k = NRD, zz = 0;
#pragma unroll
    for (int q = NRD - 1; q >= 0; --q)
    {
        const uint32_t z = haszero8(R[q] ^ cc);
        k                = z ? (uint32_t) q : k;
        zz               = z ? z : zz;
    }
    const uint32_t b    = (uint32_t) __builtin_ctz(zz | 0x80000000u) >> 3;  // 3 when not found
    const uint32_t part = b >= 3 ? 0xFFFFFFFFu : (1u << (8 * b + 8)) - 1u;  // bytes 0..b of register k
    uint32_t       rank;
    if (__builtin_amdgcn_ballot_w64(k == NRD))
        rank = k < NRD ? k * 4 + b : MTF_REG + c - count_below(R, c);
    else
        rank = k * 4 + b;
#pragma unroll
    for (int q = NRD - 1; q >= 0; --q)
    {
        const uint32_t sh = q ? __builtin_amdgcn_alignbit(R[q], R[q - 1], 24) : (R[0] << 8) | c;
        const uint32_t m  = (uint32_t) q < k ? 0xFFFFFFFFu : ((uint32_t) q == k ? part : 0u);
        R[q]              = (sh & m) | (R[q] & ~m);
    }
    return rank;
}

// The first MTF_REG entries of a segment's start table for a block of <= MTF_REG distinct symbols,
// built by one wave: the seen symbols (last occurrence >= 0, at most MTF_REG of them) ordered by
// decreasing last occurrence -- each one's position is the number of seen symbols seen later --
// then the smallest unseen byte values in increasing order.  Lane l < NRD returns dword l (entries
// 4l .. 4l+3).  Replaces a 256-key bitonic sort per segment.
__device__ __forceinline__ uint32_t start_front_small(const int32_t* __restrict__ st, uint32_t* sc_t, uint32_t* sc_c, uint8_t* sc_out)
{
    const int      lane = lane_id();
    const int4     tv   = reinterpret_cast<const int4*>(st)[lane];
    const int32_t  tt[4] = {tv.x, tv.y, tv.z, tv.w};
    uint32_t       nseen = 0, seen_before = 0, unseen_before = 0;
    uint64_t       bal[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        bal[r] = __builtin_amdgcn_ballot_w64(tt[r] >= 0);
        nseen += (uint32_t) __popcll(bal[r]);
    }
    // value c = 4 lane + r: seen values below it (lanes below, then r' < r in this lane)
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        seen_before += (uint32_t) __popcll(bal[r] & below);
    uint32_t own_seen = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        const uint32_t c = (uint32_t) lane * 4 + r;
        if (tt[r] >= 0)
        {
            const uint32_t i = seen_before + own_seen;  // index among seen values (value order)
            sc_t[i]          = (uint32_t) tt[r];
            sc_c[i]          = c;
            ++own_seen;
        }
        else
        {
            unseen_before = c - (seen_before + own_seen);  // unseen values below c
            const uint32_t pos = nseen + unseen_before;
            if (pos < MTF_REG)
                sc_out[pos] = (uint8_t) c;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if ((uint32_t) lane < nseen)
    {
        const uint32_t my = sc_t[lane];
        uint32_t       p  = 0;
        for (uint32_t j = 0; j < nseen; ++j)
            p += sc_t[j] > my ? 1u : 0u;
        sc_out[p] = (uint8_t) sc_c[lane];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t d = (lane < NRD) ? reinterpret_cast<const uint32_t*>(sc_out)[lane] : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return d;
}

// ---- position tables: blocks of <= 16 / 32 distinct values, all below 127 ----
// The table is kept inverted: byte a of NP registers holds 0x80 | position of the block's a-th
// alphabet value (input bytes are mapped to alphabet indices through an LDS copy of amap).  A
// step reads the symbol's position r, adds one to every position below r and sets the symbol's
// to 0 -- the move to front -- with byte-parallel arithmetic: bit 7 of byte (0x80 | p) - r is set
// iff p >= r (the guard bit keeps the bytes from borrowing into each other; positions stay below
// 127, so p + 1 never reaches the guard).  About 4 VALU per table dword plus a select tree, 45 / 75
// VALU per symbol for 4 / 8 dwords against ~120 for the byte table's search and shift.  Unused
// bytes hold 0xFF (never below any r, never selected).
template <int NP>
__device__ __forceinline__ uint32_t mtf_step_pos(uint32_t (&R)[NP], uint32_t a)
{
    const uint32_t q = a >> 2;
    // The table dwords as opaque scalar values, used for the select AND the update (so the barrier
    // costs no copies): a select tree over loads of one array became a dynamically indexed array
    // (the table in scratch memory).
    const auto op = [](uint32_t v) {
        asm("" : "+v"(v));
        return v;
    };
    uint32_t v[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k)
        v[k] = op(R[k]);
    uint32_t x;
    if constexpr (NP > 4)
    {
        // 5..8 dwords (17..32 values): a three-level tree, missing leaves never selected
        constexpr int  i5 = NP > 5 ? 5 : NP - 1, i6 = NP > 6 ? 6 : NP - 1, i7 = NP > 7 ? 7 : NP - 1;
        const uint32_t x0 = (q & 1) ? v[1] : v[0], x1 = (q & 1) ? v[3] : v[2];
        const uint32_t x2 = NP > 5 ? ((q & 1) ? v[i5] : v[4]) : v[4];
        const uint32_t x3 = NP > 7 ? ((q & 1) ? v[i7] : v[i6]) : v[i6];
        const uint32_t y0 = (q & 2) ? x1 : x0, y1 = NP > 6 ? ((q & 2) ? x3 : x2) : x2;
        x = (q & 4) ? y1 : y0;
    }
    else
    {
        static_assert(NP == 4, "4 to 8 table dwords");
        const uint32_t x0 = (q & 1) ? v[1] : v[0], x1 = (q & 1) ? v[3] : v[2];
        x = (q & 2) ? x1 : x0;
    }
    const uint32_t sh = (a & 3u) << 3;
    const uint32_t r  = (x >> sh) & 0x7Fu;
    const uint32_t rr = __builtin_amdgcn_perm(0u, r, 0x00000000u);  // r in every byte
    const uint32_t dl = r << sh;
#pragma unroll
    for (int k = 0; k < NP; ++k)
    {
        // bit 7 of byte (0x80 | p) - r is clear iff p < r: those positions move up by one
        const uint32_t ge = (v[k] - rr) >> 7;
        uint32_t       inc;  // ~ge & 0x01010101 in one v_bfi (the compiler emits a not and an and)
        asm("v_bfi_b32 %0, %1, 0, %2" : "=v"(inc) : "v"(ge), "s"(0x01010101u));
        const uint32_t nv  = v[k] + inc;
        R[k]               = ((uint32_t) k == q) ? nv - dl : nv;
    }
    return r;
}

// Symbols and ranks move through LDS in rounds of 64 bytes per segment, chunk-major (io[c][t]:
// the 16-byte accesses of consecutive threads are conflict-free): the workgroup loads the next 64
// bytes of all its segments with line-contiguous 16-byte loads (4 lanes per 64-byte run), every
// thread codes its own 64 symbols in place, and the workgroup stores them back the same way.  Each
// thread reading its own segment 16 bytes at a time from HBM (1 KiB apart from its neighbours) moved
// 2.8 GB per 256 MiB step for 0.5 GB of data.
constexpr uint32_t MR_RB = 64;           // bytes per segment per round
constexpr uint32_t MR_NC = MR_RB / 16;   // 16-byte chunks per segment per round

// The coding loop of one workgroup iteration (STEP: one MTF step on the thread's table R).
template <int NR, bool MAP, typename Step>
__device__ __forceinline__ void mtf_code_rounds(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t (&R)[NR], uint4 (*io)[TPB],
                                                const uint64_t* s_off, const uint32_t* s_len, const uint8_t* map_s, Step step)
{
    const uint32_t t    = threadIdx.x;
    const uint32_t len  = s_len[t];
    const uint64_t off  = s_off[t];
    const uint32_t full = len & ~15u;  // whole 16-byte chunks go through LDS, the tail byte by byte
    uint32_t       rmax = 0;           // rounds the workgroup needs
    for (uint32_t u = 0; u < TPB; ++u)
        rmax = max(rmax, (s_len[u] & ~15u));
    for (uint32_t r0 = 0; r0 < rmax; r0 += MR_RB)
    {
        // load: piece p = (segment p / MR_NC, chunk p % MR_NC)
#pragma unroll
        for (uint32_t i = 0; i < MR_NC; ++i)
        {
            const uint32_t p = t + i * TPB, sl = p / MR_NC, c = p % MR_NC;
            const uint32_t at = r0 + c * 16;
            if (at + 16 <= (s_len[sl] & ~15u))
            {
                const uint8_t* q = in + s_off[sl] + at;
                if ((((uintptr_t) q) & 15) == 0)
                    io[c][sl] = *reinterpret_cast<const uint4*>(q);
                else
                {
                    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int k = 0; k < 16; ++k)
                        w[k >> 2] |= (uint32_t) q[k] << (8 * (k & 3));
                    io[c][sl] = make_uint4(w[0], w[1], w[2], w[3]);
                }
            }
        }
        __syncthreads();
#pragma unroll 1
        for (uint32_t c = 0; c < MR_NC && r0 + c * 16 < full; ++c)
        {
            uint4 cur = io[c][t];
            if (MAP)
            {
                // input bytes -> alphabet indices (16 independent LDS lookups)
                uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w}, m[4] = {0, 0, 0, 0};
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    m[k >> 2] |= (uint32_t) map_s[(w[k >> 2] >> (8 * (k & 3))) & 0xFFu] << (8 * (k & 3));
                cur = make_uint4(m[0], m[1], m[2], m[3]);
            }
            // 16 symbols, a dword (4 steps, constant byte positions) per iteration of a rolled loop
            // over a 4-dword queue (16 inlined steps cost 2x the registers for nothing, the steps
            // are serial; a 128-bit shift register cost 8 VALU of shifts per symbol)
            uint32_t q0 = cur.x, q1 = cur.y, q2 = cur.z, q3 = cur.w, o0 = 0, o1 = 0, o2 = 0, o3 = 0;
#pragma unroll 1
            for (int j = 0; j < 4; ++j)
            {
                const uint32_t w  = q0;
                const uint32_t k0 = step(R, w & 0xFFu);
                const uint32_t k1 = step(R, (w >> 8) & 0xFFu);
                const uint32_t k2 = step(R, (w >> 16) & 0xFFu);
                const uint32_t k3 = step(R, w >> 24);
                q0 = q1, q1 = q2, q2 = q3;
                o0 = o1, o1 = o2, o2 = o3;
                o3 = k0 | (k1 << 8) | (k2 << 16) | (k3 << 24);
            }
            io[c][t] = make_uint4(o0, o1, o2, o3);
        }
        __syncthreads();
#pragma unroll
        for (uint32_t i = 0; i < MR_NC; ++i)
        {
            const uint32_t p = t + i * TPB, sl = p / MR_NC, c = p % MR_NC;
            const uint32_t at = r0 + c * 16;
            if (at + 16 <= (s_len[sl] & ~15u))
            {
                uint8_t*    q = out + s_off[sl] + at;
                const uint4 v = io[c][sl];
                if ((((uintptr_t) q) & 15) == 0)
                    *reinterpret_cast<uint4*>(q) = v;
                else
                {
                    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int k = 0; k < 16; ++k)
                        q[k] = (uint8_t) (w[k >> 2] >> (8 * (k & 3)));
                }
            }
        }
        __syncthreads();
    }
    for (uint32_t i = full; i < len; ++i)
        out[off + i] = (uint8_t) step(R, MAP ? (uint32_t) map_s[in[off + i]] : (uint32_t) in[off + i]);
}

// Position-table blocks (amode 4 / 8), one thread per 512-byte half segment (twice the chains of
// one thread per segment: the coding loop is a dependent chain per symbol, and at one segment per
// thread a 256 MiB batch had only 4 waves per SIMD to overlap them).  Workgroup (x, y) codes half
// segments [256 x, 256 x + 256) of block y, so the block's alphabet map sits in LDS and its table
// width (4 dwords for <= 16 values, else 8) is uniform; each thread starts from its half segment's
// position table (k_mtf_scan).
template <int NP>
__device__ __forceinline__ void encode_pos_wg(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, const int32_t* __restrict__ state,
                                              uint32_t s, uint32_t half, uint32_t len, uint4 (*io)[TPB], const uint64_t* s_off,
                                              const uint32_t* s_len, const uint8_t* map_s)
{
    uint32_t R[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k)
        R[k] = 0xFFFFFFFFu;
    if (len)
    {
        const uint4* pt = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(state) + (size_t) s * 1024 + 512 + half * 32);
        const uint4  v0 = pt[0];
        const uint4  v1 = NP > 4 ? pt[1] : v0;
        const uint32_t t8[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int k = 0; k < NP; ++k)
            R[k] = t8[k];
    }
    mtf_code_rounds<NP, true>(in, out, R, io, s_off, s_len, map_s, [](uint32_t (&T)[NP], uint32_t a) { return mtf_step_pos<NP>(T, a); });
}

__global__ void __launch_bounds__(TPB, 8) k_mtf_encode_pos(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, const Piece* __restrict__ segs,
                                                        const uint32_t* __restrict__ first_seg, const uint32_t* __restrict__ nseg_blk,
                                                        uint32_t nblocks, const int32_t* __restrict__ state, const uint8_t* __restrict__ amap,
                                                        const uint32_t* __restrict__ amode)
{
    __shared__ uint4    io[MR_NC][TPB];
    __shared__ uint64_t s_off[TPB];
    __shared__ uint32_t s_len[TPB];  // 0: past the block
    __shared__ uint8_t  map_s[256];
    const uint32_t t = threadIdx.x;
    for (uint32_t b = blockIdx.y; b < nblocks; b += gridDim.y)
    {
        const uint32_t mode = amode[b], nh = 2 * nseg_blk[b], h = blockIdx.x * TPB + t;
        if (mode == 0 || blockIdx.x * TPB >= nh)
            continue;  // uniform per workgroup
        const uint32_t s   = first_seg[b] + (h >> 1), half = h & 1u;
        uint32_t       len = 0;
        uint64_t       off = 0;
        if (h < nh)
        {
            const Piece    P  = segs[s];
            const uint32_t lo = half * (MTF_SEG_ENC / 2);
            if (P.len > lo)
            {
                len = min(MTF_SEG_ENC / 2, P.len - lo);
                off = P.off + lo;
            }
        }
        s_off[t] = off;
        s_len[t] = len;
        map_s[t] = amap[(size_t) b * 256 + t];
        __syncthreads();
        switch (mode)  // table dwords: ceil(values / 4), uniform per block
        {
        case 4: encode_pos_wg<4>(in, out, state, s, half, len, io, s_off, s_len, map_s); break;
        case 5: encode_pos_wg<5>(in, out, state, s, half, len, io, s_off, s_len, map_s); break;
        case 6: encode_pos_wg<6>(in, out, state, s, half, len, io, s_off, s_len, map_s); break;
        case 7: encode_pos_wg<7>(in, out, state, s, half, len, io, s_off, s_len, map_s); break;
        default: encode_pos_wg<8>(in, out, state, s, half, len, io, s_off, s_len, map_s); break;
        }
        __syncthreads();
    }
}

// Other blocks of at most MTF_REG distinct symbols: one thread per segment with the byte tables
// (mtf_step_reg).
__global__ void __launch_bounds__(TPB) k_mtf_encode_reg(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, const Piece* __restrict__ segs,
                                                        uint32_t nseg, const int32_t* __restrict__ state, const uint32_t* __restrict__ nsym,
                                                        const uint32_t* __restrict__ amode)
{
    __shared__ uint32_t front[NRD][TPB];  // start-table fronts of the workgroup's segments (thread-major: conflict-free)
    __shared__ uint32_t sc_t[TPB / 64][MTF_REG], sc_c[TPB / 64][MTF_REG];
    __shared__ __attribute__((aligned(4))) uint8_t sc_out[TPB / 64][MTF_REG];
    __shared__ uint4    io[MR_NC][TPB];
    __shared__ uint64_t s_off[TPB];
    __shared__ uint32_t s_len[TPB];  // 0: not coded by this kernel (or past the batch)
    const uint32_t t    = threadIdx.x;
    const int      lane = lane_id();
    const uint32_t wave = t >> 6;
    for (uint32_t g0 = blockIdx.x * TPB; g0 < nseg; g0 += gridDim.x * TPB)
    {
        const auto mine = [&](const Piece& P) { return nsym[P.block] <= MTF_REG && amode[P.block] == 0; };
        {
            const uint32_t s = g0 + t;
            uint32_t       l = 0;
            if (s < nseg)
            {
                const Piece P = segs[s];
                s_off[t]      = P.off;
                l             = mine(P) ? P.len : 0u;
            }
            s_len[t] = l;
        }
        if (!__syncthreads_or(s_len[t] != 0))
            continue;
        for (int q = 0; q < 64; ++q)
        {
            const uint32_t owner = wave * 64 + q;
            const uint32_t s     = g0 + owner;
            if (s >= nseg)
                break;
            const Piece P = segs[s];
            if (!mine(P))
                continue;
            const uint32_t d = (P.start == 0) ? (uint32_t) (lane * 4) * 0x01010101u + 0x03020100u
                                              : start_front_small(state + (size_t) s * 256, sc_t[wave], sc_c[wave], sc_out[wave]);
            if (lane < NRD)
                front[lane][owner] = d;
        }
        __syncthreads();
        const bool act = s_len[t] != 0;
        uint32_t   R[NRD];
#pragma unroll
        for (int k = 0; k < NRD; ++k)
            R[k] = act ? front[k][t] : 0u;
        mtf_code_rounds<NRD, false>(in, out, R, io, s_off, s_len, nullptr, [](uint32_t (&T)[NRD], uint32_t c) { return mtf_step_reg(T, c); });
        __syncthreads();
    }
}

// ---- wave-cooperative MTF: blocks of more than MTF_REG distinct symbols ----
// One wave codes one segment (staged in LDS, ranks written back in place), 64 symbols at a time,
// one per lane, from the table at the start of the 64-symbol chunk: list[p] = symbol at position p
// and pos[c] = position of symbol c (256-byte LDS rows per wave).  The table lists symbols by
// decreasing last-occurrence time, so the rank of lane i's symbol s is the number of symbols whose
// last occurrence before i is later than s's:
//   * s occurred earlier in the chunk, last at lane j ("repeat"): the distinct symbols of lanes
//     (j, i) = #{k in (j, i): nxt_k >= i} (nxt_k = next lane holding s_k, 64 if none);
//   * otherwise ("first"): pos[s] plus the chunk's distinct symbols before i that stood behind s,
//     pos[s] + #{k in F, k < i} - #{k in F, k < i: pos_k < pos[s]} over the first lanes F.
// The first count is bit-sliced: one ballot per key bit and a few 64-bit mask operations per lane
// (v_bitop3 on gfx950).  Repeats are few in high-entropy data (about 7 of 64 in uniform random
// bytes), so they are counted one at a time with a ballot each unless there are many.  Then the
// table moves: the chunk's distinct symbols take the front by decreasing last occurrence and the
// other entries keep their order behind them (a wave compaction of the list).  The cost does not
// depend on the ranks (uniform random data: ranks average 127.5).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t ballot64(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// bit b of x as an all-zeros / all-ones word (v_bfe_i32)
__device__ __forceinline__ uint32_t bitmask(uint32_t x, int b) { return (uint32_t) (((int32_t) (x << (31 - b))) >> 31); }

// #{k in dom : key_k < q} for this lane's query q (keys and queries of NB bits): walk the bits from
// the top keeping E = the lanes of dom whose key agrees with q on the bits above; the lanes that
// first differ at bit b with key bit 0 < query bit 1 are below q.  (32-bit halves, so that each
// update is one v_bitop3 with the ballot as its scalar operand.)
template <int NB>
__device__ __forceinline__ uint32_t count_less(uint32_t key, uint32_t q, uint64_t dom)
{
    uint32_t el = (uint32_t) dom, eh = (uint32_t) (dom >> 32), ll = 0, lh = 0;
#pragma unroll
    for (int b = NB - 1; b >= 0; --b)
    {
        const uint64_t B  = ballot64(bitmask(key, b) != 0);
        const uint32_t bl = (uint32_t) B, bh = (uint32_t) (B >> 32);
        const uint32_t mq = bitmask(q, b);
        ll |= el & ~bl & mq;
        lh |= eh & ~bh & mq;
        el &= ~(bl ^ mq);
        eh &= ~(bh ^ mq);
    }
    return (uint32_t) __popc(ll) + (uint32_t) __popc(lh);
}

constexpr int MTF_REP_LOOP = 4;  // repeats in a 64-symbol chunk counted one ballot each up to this many (random data: 0/4/8/16 -> 2.05/2.04/2.05/2.20 ms)
static_assert(MTF_SEG_ENC == 1024, "k_mtf_encode_wave stages a segment as 64 lanes x 16 bytes");

__global__ void __launch_bounds__(TPB) k_mtf_encode_wave(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, const Piece* __restrict__ segs,
                                                         uint32_t nseg, const int32_t* __restrict__ state, const uint32_t* __restrict__ nsym)
{
    __shared__ uint32_t pos_s[TPB / 64][64];   // byte c of a wave's row: table position of symbol c
    __shared__ uint32_t list_s[TPB / 64][64];  // byte p: symbol at table position p
    __shared__ uint32_t mark_s[TPB / 64][64];  // byte p != 0: position p holds a symbol of the chunk
    __shared__ uint4    buf_s[TPB / 64][64];   // the segment: symbols, overwritten by their ranks
    const int      lane  = lane_id();
    const uint32_t wave  = wave_id();
    uint8_t*       pos   = reinterpret_cast<uint8_t*>(pos_s[wave]);
    uint8_t*       list  = reinterpret_cast<uint8_t*>(list_s[wave]);
    uint8_t*       mark  = reinterpret_cast<uint8_t*>(mark_s[wave]);
    uint8_t*       buf   = reinterpret_cast<uint8_t*>(buf_s[wave]);
    const uint64_t below = (1ull << lane) - 1ull;
    const uint64_t above = ~below << 1;
    mark_s[wave][lane]   = 0;
    for (uint32_t s = blockIdx.x * (TPB / 64) + wave; s < nseg; s += gridDim.x * (TPB / 64))
    {
        const Piece P = segs[s];
        if (nsym[P.block] <= MTF_REG)
            continue;
        const bool full = P.len == MTF_SEG_ENC && ((P.off & 15) == 0);
        if (full)
            buf_s[wave][lane] = reinterpret_cast<const uint4*>(in + P.off)[lane];
        else
            for (uint32_t i = lane; i < P.len; i += 64)
                buf[i] = in[P.off + i];
        {
            const uint32_t d = (P.start == 0) ? (uint32_t) (lane * 4) * 0x01010101u + 0x03020100u
                                              : start_table_dword(state + (size_t) s * 256);  // symbols at positions 4 lane + r
            list_s[wave][lane] = d;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                pos[(d >> (8 * r)) & 0xFF] = (uint8_t) (lane * 4 + r);
        }
        wave_lds_sync();
        for (uint32_t c0 = 0; c0 < P.len; c0 += 64)
        {
            const uint32_t nv    = min(64u, P.len - c0);
            const bool     valid = (uint32_t) lane < nv;
            const uint32_t sym   = valid ? buf[c0 + lane] : 0u;
            const uint64_t V     = ballot64(valid);
            uint32_t       el = (uint32_t) V, eh = (uint32_t) (V >> 32);  // lanes holding the same symbol
#pragma unroll
            for (int b = 0; b < 8; ++b)
            {
                const uint32_t m = bitmask(sym, b);
                const uint64_t B = ballot64(m != 0);
                el &= ~((uint32_t) B ^ m);
                eh &= ~((uint32_t) (B >> 32) ^ m);
            }
            const uint64_t eq  = ((uint64_t) eh << 32) | el;
            const uint64_t pm  = eq & below, nm = eq & above;
            const int      j   = pm ? 63 - __builtin_clzll(pm) : -1;
            const uint32_t nxt = nm ? (uint32_t) __builtin_ctzll(nm) : 64u;
            const uint32_t p0  = pos[sym];
            const bool     rep = j >= 0;
            const uint64_t Fm  = V & ~ballot64(rep);  // first occurrences
            const uint64_t Am  = V & ~Fm;             // repeats
            uint32_t       rank = 0;
            if (Fm)
            {
                const uint64_t fb = Fm & below;
                rank              = p0 + (uint32_t) __popcll(fb) - count_less<8>(p0, p0, fb);
            }
            if (__popcll(Am) > MTF_REP_LOOP)
            {
                // many repeats: #{k in (j, i): nxt_k < i}, nxt in [1, 64] -> 7 bits
                const uint64_t in_ji = below & (rep ? ~((2ull << j) - 1ull) : 0ull);
                const uint32_t ra    = (uint32_t) (lane - j - 1) - count_less<7>(nxt, (uint32_t) lane, in_ji);
                if (rep)
                    rank = ra;
            }
            else
            {
                uint64_t A = Am;
                while (A)
                {
                    const int i = __builtin_ctzll(A);
                    A &= A - 1;
                    const int      ji = __builtin_amdgcn_readlane(j, i);
                    const uint64_t G  = ballot64(nxt >= (uint32_t) i) & ((1ull << i) - 1ull) & ~((2ull << ji) - 1ull);
                    rank              = lane == i ? (uint32_t) __popcll(G) : rank;
                }
            }
            if (valid)
                buf[c0 + lane] = (uint8_t) rank;
            // move the chunk's symbols to the front: they take positions 0 .. Dc-1 by decreasing last
            // occurrence, the other entries keep their order behind them
            const bool     last = valid && nxt == 64u;
            const uint64_t Lm   = ballot64(last);
            const uint32_t Dc   = (uint32_t) __popcll(Lm);
            if (last)
                mark[p0] = 1;
            wave_lds_sync();
            const uint32_t mw = mark_s[wave][lane];  // positions 4 lane .. 4 lane + 3
            const uint32_t lw = list_s[wave][lane];
            uint32_t       kept[4], nk = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                kept[r] = ((mw >> (8 * r)) & 0xFF) ? 0u : 1u;
                nk += kept[r];
            }
            uint32_t ex;
            (void) wave_scan<true>(nk, 0u, OpAdd(), &ex);
            wave_lds_sync();
            mark_s[wave][lane] = 0;
            uint32_t o = Dc + ex;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (kept[r])
                {
                    const uint32_t c = (lw >> (8 * r)) & 0xFF;
                    list[o]          = (uint8_t) c;
                    pos[c]           = (uint8_t) o;
                    ++o;
                }
            if (last)
            {
                const uint32_t np = (uint32_t) __popcll(Lm & above);
                list[np]          = (uint8_t) sym;
                pos[sym]          = (uint8_t) np;
            }
            wave_lds_sync();
        }
        if (full)
            reinterpret_cast<uint4*>(out + P.off)[lane] = buf_s[wave][lane];
        else
            for (uint32_t i = lane; i < P.len; i += 64)
                out[P.off + i] = buf[i];
        wave_lds_sync();
    }
}

// ------------------------------------------------------------------------------------------------
// decode
// ------------------------------------------------------------------------------------------------
// Pass 1: decode each segment from the identity table (labels -> lab, end table -> perm), with the
// table front (entries 0..15) in four registers and entries 16..255 in 15 LDS chunks of 16 bytes, chunk-major (tb[k * TPB + t]: the
// 16-byte accesses of consecutive lanes are conflict-free).  A step at rank r reads its symbol
// straight from the register or chunk holding position r, then shifts the positions below r up by
// one, 16 at a time; post-BWT ranks are small, so most steps touch registers only.  Input and
// labels move 16 bytes at a time, the next 16 input bytes loaded before the current ones decode.
__device__ __forceinline__ uint4 shift_chunk(const uint4& v, uint32_t& top)
{
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    uint32_t       o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
        const uint32_t ntop = d[q] >> 24;
        o[q]                = shift1(d[q], top);
        top                 = ntop;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

__device__ __forceinline__ uint4 shift_chunk_upto(const uint4& v, uint32_t top, uint32_t rr)
{
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    const uint32_t k = rr >> 2, b = rr & 3;
    uint32_t       o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
        const uint32_t ntop = d[q] >> 24;
        o[q]                = ((uint32_t) q < k) ? shift1(d[q], top) : ((uint32_t) q == k) ? shift_upto(d[q], top, b) : d[q];
        top                 = ntop;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, uint32_t i)
{
    const uint32_t q = i >> 2;
    const uint32_t d = q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
    return (d >> (8 * (i & 3))) & 0xFF;
}

__device__ __forceinline__ uint32_t dec_step(uint32_t (&R)[4], uint4* tb, uint32_t t, uint32_t r)
{
    if (r < 16)
    {
        const uint32_t k = r >> 2, b = r & 3;
        const uint32_t c = ((k == 0 ? R[0] : k == 1 ? R[1] : k == 2 ? R[2] : R[3]) >> (8 * b)) & 0xFF;
        uint32_t       top = c;
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {
            const uint32_t cur = R[q], ntop = cur >> 24;
            if ((uint32_t) q < k)
                R[q] = shift1(cur, top);
            else if ((uint32_t) q == k)
                R[q] = shift_upto(cur, top, b);
            top = ntop;
        }
        return c;
    }
    const uint32_t ch = r >> 4, rr = r & 15;
    const uint4    v  = tb[(ch - 1) * TPB + t];
    const uint32_t c  = byte_of(v, rr);
    uint32_t       top = c;
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
        const uint32_t cur = R[q], ntop = cur >> 24;
        R[q]                = shift1(cur, top);
        top                 = ntop;
    }
    for (uint32_t k = 1; k < ch; ++k)
    {
        const uint4 u            = tb[(k - 1) * TPB + t];
        tb[(k - 1) * TPB + t]    = shift_chunk(u, top);
    }
    tb[(ch - 1) * TPB + t] = shift_chunk_upto(v, top, rr);
    return c;
}

__global__ void __launch_bounds__(TPB) k_mtf_dec_local2(const uint8_t* __restrict__ in, uint8_t* __restrict__ lab,
                                                        const Piece* __restrict__ segs, uint32_t nseg, uint32_t* __restrict__ perm)
{
    extern __shared__ __attribute__((aligned(16))) uint4 tb[];  // 15 * TPB chunks
    const uint32_t t = threadIdx.x;
    for (uint32_t g0 = blockIdx.x * TPB; g0 < nseg; g0 += gridDim.x * TPB)
    {
        const uint32_t s = g0 + t;
        if (s >= nseg)
            continue;
        uint32_t R[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            R[q] = (uint32_t) (q * 4) * 0x01010101u + 0x03020100u;
        for (uint32_t k = 1; k < 16; ++k)
        {
            const uint32_t b0 = k * 16;
            tb[(k - 1) * TPB + t] = make_uint4(b0 * 0x01010101u + 0x03020100u, (b0 + 4) * 0x01010101u + 0x03020100u,
                                               (b0 + 8) * 0x01010101u + 0x03020100u, (b0 + 12) * 0x01010101u + 0x03020100u);
        }
        const Piece    P   = segs[s];
        const uint8_t* src = in + P.off;
        uint8_t*       dst = lab + P.off;
        uint32_t       i   = 0;
        if ((((uintptr_t) src | (uintptr_t) dst) & 15) == 0 && P.len >= 16)
        {
            const uint32_t nv  = P.len / 16;
            uint4          nxt = reinterpret_cast<const uint4*>(src)[0];
            for (uint32_t v = 0; v < nv; ++v)
            {
                const uint4 cur = nxt;
                if (v + 1 < nv)
                    nxt = reinterpret_cast<const uint4*>(src)[v + 1];
                // 16 ranks shifted out of a 128-bit register pair, labels shifted in (rolled: the steps are serial)
                uint64_t ilo = ((uint64_t) cur.y << 32) | cur.x, ihi = ((uint64_t) cur.w << 32) | cur.z;
                uint64_t olo = 0, ohi = 0;
#pragma unroll 1
                for (int j = 0; j < 16; ++j)
                {
                    const uint32_t c = dec_step(R, tb, t, (uint32_t) ilo & 0xFFu);
                    ilo              = (ilo >> 8) | (ihi << 56);
                    ihi >>= 8;
                    olo = (olo >> 8) | (ohi << 56);
                    ohi = (ohi >> 8) | ((uint64_t) c << 56);
                }
                reinterpret_cast<uint4*>(dst)[v] = make_uint4((uint32_t) olo, (uint32_t) (olo >> 32), (uint32_t) ohi, (uint32_t) (ohi >> 32));
            }
            i = nv * 16;
        }
        for (; i < P.len; ++i)
            dst[i] = (uint8_t) dec_step(R, tb, t, src[i]);
        uint32_t* pm = perm + (size_t) s * 64;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            pm[q] = R[q];
        for (uint32_t k = 1; k < 16; ++k)
        {
            const uint4 u = tb[(k - 1) * TPB + t];
            pm[k * 4 + 0] = u.x;
            pm[k * 4 + 1] = u.y;
            pm[k * 4 + 2] = u.z;
            pm[k * 4 + 3] = u.w;
        }
    }
}

// Pass 2: one wave per block composes start tables S_{k+1}[j] = S_k[P_k[j]] (in place in perm:
// perm[k] becomes S_k).
__global__ void __launch_bounds__(64) k_mtf_dec_compose(const uint32_t* __restrict__ first_seg, const uint32_t* __restrict__ nseg_blk,
                                                        uint32_t nblocks, uint32_t* __restrict__ perm)
{
    const int lane = lane_id();
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint32_t s0 = first_seg[b], ns = nseg_blk[b];
        uint32_t       S  = (uint32_t) (lane * 4) * 0x01010101u + 0x03020100u;  // identity
        uint32_t       Pn = perm[(size_t) s0 * 64 + lane];
        for (uint32_t k = 0; k < ns; ++k)
        {
            const uint32_t Pk = Pn;
            if (k + 1 < ns)
                Pn = perm[(size_t) (s0 + k + 1) * 64 + lane];
            perm[(size_t) (s0 + k) * 64 + lane] = S;
            uint32_t nS = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const uint32_t j   = (Pk >> (8 * r)) & 0xFF;
                const uint32_t src = __shfl(S, (int) (j >> 2), 64);
                nS |= ((src >> (8 * (j & 3))) & 0xFF) << (8 * r);
            }
            S = nS;
        }
    }
}

// Pass 3: out = S_k[label]
__global__ void __launch_bounds__(TPB) k_mtf_dec_relabel(const uint8_t* __restrict__ lab, uint8_t* __restrict__ out,
                                                         const Piece* __restrict__ segs, uint32_t nseg, const uint32_t* __restrict__ perm)
{
    __shared__ uint8_t S[256];
    for (uint32_t s = blockIdx.x; s < nseg; s += gridDim.x)
    {
        if (threadIdx.x < 64)
            reinterpret_cast<uint32_t*>(S)[threadIdx.x] = perm[(size_t) s * 64 + threadIdx.x];
        __syncthreads();
        const Piece P = segs[s];
        // 8 bytes per thread and round where the segment is 8-aligned (MTF_SEG = 2048 = 256 x 8:
        // one round; a byte per thread cost an instruction per byte)
        uint32_t done = 0;
        if ((P.off & 7u) == 0)
        {
            done = P.len & ~7u;
            for (uint32_t i = threadIdx.x * 8; i < done; i += TPB * 8)
            {
                const uint2 v = *reinterpret_cast<const uint2*>(lab + P.off + i);
                uint32_t    o[2];
#pragma unroll
                for (int h = 0; h < 2; ++h)
                {
                    const uint32_t x = h ? v.y : v.x;
                    o[h] = (uint32_t) S[x & 0xFFu] | ((uint32_t) S[(x >> 8) & 0xFFu] << 8) | ((uint32_t) S[(x >> 16) & 0xFFu] << 16) |
                           ((uint32_t) S[x >> 24] << 24);
                }
                *reinterpret_cast<uint2*>(out + P.off + i) = make_uint2(o[0], o[1]);
            }
        }
        for (uint32_t i = done + threadIdx.x; i < P.len; i += TPB)
            out[P.off + i] = S[lab[P.off + i]];
        __syncthreads();
    }
}

}  // namespace

bool mtf_encode_device(MtfWorkspace& w, const uint8_t* d_in, uint8_t* d_out, const BlockDesc* h_blocks, uint32_t nblocks, hipStream_t s,
                       const uint32_t* d_amask)
{
    if (!w.tiling.build(h_blocks, nblocks, MTF_SEG_ENC, s))
        return false;
    const uint32_t nseg = w.tiling.n;
    if (!w.reserve((size_t) nseg * 256 * 4) || !w.reserve_blocks(nblocks))
        return false;
    int32_t* st = reinterpret_cast<int32_t*>(w.state);
    {
        BRA_PROF(P_MTF_LASTOCC, s);
        if (!d_amask)
        {
            BRA_HIP_CHECK(hipMemsetAsync(w.amask, 0, (size_t) nblocks * 32, s));
            hipLaunchKernelGGL(k_mtf_presence, dim3(std::min<uint32_t>(div_up(nseg, TPB / 64), 16384)), dim3(TPB), 0, s, d_in, w.tiling.d_pieces, nseg,
                               w.amask);
            d_amask = w.amask;
        }
        hipLaunchKernelGGL(k_mtf_alpha, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(TPB), 0, s, d_amask, nblocks, w.nsym, w.amap, w.ainv, w.amode);
        hipLaunchKernelGGL(k_mtf_lastocc, dim3(std::min<uint32_t>(div_up(nseg, TPB / 64), 16384)), dim3(TPB), 0, s, d_in, w.tiling.d_pieces, nseg, st,
                           w.amode, w.nsym, w.ainv);
    }
    if (w.pt_key != w.tiling.h_count)
    {
        // chunk geometry of the position-table passes (host-built once per geometry)
        std::vector<uint32_t> c0(nblocks), cb;
        for (uint32_t b = 0; b < nblocks; ++b)
        {
            c0[b] = (uint32_t) cb.size();
            cb.insert(cb.end(), div_up(2ull * w.tiling.h_count[b], PT_CHUNK), b);
        }
        const uint32_t nc = (uint32_t) cb.size();
        w.pt_key.clear();
        if (nblocks > w.pt_cap_b)
        {
            w.pt_cap_b = 0;
            if (!dev_alloc(w.pt_chunk0, (uint64_t) nblocks + 64))
                return false;
            w.pt_cap_b = nblocks + 64;
        }
        if (nc + 1 > w.pt_cap_c)
        {
            w.pt_cap_c = 0;
            if (!dev_alloc(w.pt_chunk_blk, (uint64_t) nc + 64) || !dev_alloc(w.pt_cmax, 32ull * (nc + 64)))
                return false;
            w.pt_cap_c = nc + 64;
        }
        BRA_HIP_CHECK(hipMemcpyAsync(w.pt_chunk0, c0.data(), (size_t) nblocks * 4, hipMemcpyHostToDevice, s));
        if (nc)
            BRA_HIP_CHECK(hipMemcpyAsync(w.pt_chunk_blk, cb.data(), (size_t) nc * 4, hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipStreamSynchronize(s));  // host vectors are the copies' sources
        w.pt_nchunks = nc;
        w.pt_key     = w.tiling.h_count;
    }
    {
        BRA_PROF(P_MTF_SCAN, s);
        hipLaunchKernelGGL(k_mtf_scan, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(TPB), 0, s, w.tiling.d_first, w.tiling.d_count,
                           nblocks, st, w.nsym, w.ainv, w.amode);
        const PtGeo    g{w.tiling.d_first, w.tiling.d_count, w.pt_chunk0, w.pt_chunk_blk, w.pt_nchunks};
        const uint32_t gc = std::max<uint32_t>(1, std::min<uint32_t>(div_up(w.pt_nchunks, TPB / 32), 16384));
        hipLaunchKernelGGL(k_mtf_pt_max, dim3(gc), dim3(TPB), 0, s, st, g, w.amode, w.pt_cmax);
        hipLaunchKernelGGL(k_mtf_pt_scan, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(TPB), 0, s, g, nblocks, w.amode, w.pt_cmax);
        hipLaunchKernelGGL(k_mtf_pt_tables, dim3(gc), dim3(TPB), 0, s, st, g, w.amode, w.nsym, w.ainv, w.pt_cmax);
    }
    {
        BRA_PROF(P_MTF_ENCODE, s);
        // every segment goes to exactly one of the three kernels (by its block's alphabet)
        uint32_t maxc = 0;
        for (uint32_t c : w.tiling.h_count)
            maxc = std::max(maxc, c);
        hipLaunchKernelGGL(k_mtf_encode_pos, dim3(div_up(2ull * maxc, TPB), std::min<uint32_t>(nblocks, 65535)), dim3(TPB), 0, s, d_in, d_out,
                           w.tiling.d_pieces, w.tiling.d_first, w.tiling.d_count, nblocks, st, w.amap, w.amode);
        hipLaunchKernelGGL(k_mtf_encode_reg, dim3(std::min<uint32_t>(div_up(nseg, TPB), 4096)), dim3(TPB), 0, s, d_in, d_out,
                           w.tiling.d_pieces, nseg, st, w.nsym, w.amode);
        hipLaunchKernelGGL(k_mtf_encode_wave, dim3(std::min<uint32_t>(div_up(nseg, TPB / 64), 16384)), dim3(TPB), 0, s, d_in, d_out,
                           w.tiling.d_pieces, nseg, st, w.nsym);
    }
    uint64_t N = 0;
    for (uint32_t b = 0; b < nblocks; ++b)
        N += h_blocks[b].len;
    prof_bytes(P_MTF_LASTOCC, (double) N + 1024.0 * nseg);
    prof_bytes(P_MTF_SCAN, 2048.0 * nseg);
    prof_bytes(P_MTF_ENCODE, 2.0 * N + 1024.0 * nseg);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

bool mtf_decode_device(MtfWorkspace& w, const uint8_t* d_in, uint8_t* d_out, uint8_t* d_tmp, const BlockDesc* h_blocks, uint32_t nblocks,
                       hipStream_t s)
{
    if (!w.tiling.build(h_blocks, nblocks, MTF_SEG, s))
        return false;
    const uint32_t nseg = w.tiling.n;
    if (!w.reserve((size_t) nseg * 256))
        return false;
    uint32_t*    perm = reinterpret_cast<uint32_t*>(w.state);
    const size_t lds  = 15 * TPB * 16;
    static bool  attr = false;
    if (!attr)
    {
        BRA_HIP_CHECK(hipFuncSetAttribute((const void*) k_mtf_dec_local2, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
        attr = true;
    }
    {
        BRA_PROF(P_DEC_MTF_LOCAL, s);
        if (g_prof)
        {
            double n = 0;  // algorithmic bytes: ranks read, labels written
            for (uint32_t b = 0; b < nblocks; ++b)
                n += h_blocks[b].len;
            prof_bytes(P_DEC_MTF_LOCAL, 2.0 * n);
        }
        hipLaunchKernelGGL(k_mtf_dec_local2, dim3(std::min<uint32_t>(div_up(nseg, TPB), 4096)), dim3(TPB), lds, s, d_in, d_tmp,
                           w.tiling.d_pieces, nseg, perm);
    }
    hipLaunchKernelGGL(k_mtf_dec_compose, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(64), 0, s, w.tiling.d_first, w.tiling.d_count,
                       nblocks, perm);
    hipLaunchKernelGGL(k_mtf_dec_relabel, dim3(std::min<uint32_t>(nseg, 16384)), dim3(TPB), 0, s, d_tmp, d_out, w.tiling.d_pieces, nseg,
                       perm);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace bra
