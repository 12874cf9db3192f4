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
//   level >= 1   MSD radix passes on the next key byte for buckets larger than a workgroup job,
//                with the key re-gathered from the input every 8 bytes.  Sub-buckets of
//                <= JOB_MAX elements are packed into wave jobs, larger ones up to 256 * waves
//                become workgroup jobs.  The host passes every count a kernel needs (tile counts,
//                list lengths) as kernel arguments; no kernel re-reads a counter another kernel
//                updated with atomics.
//   jobs         a wave (<= 256 elements) or a workgroup (<= 256 * waves) sorts in registers
//                (bitonic, 4 per lane) on 128-bit keys: group id in the top bits, then 15 (wave)
//                or 14 (workgroup) rotation bytes gathered at the group's depth.  Groups still tied
//                are compacted and re-sorted on the next bytes until no ties remain, the depth
//                reaches n (ties are then identical rotations), or a depth cap sends the group to
//                the fallback.  Job lists are reordered block-major per XCD so the gathers of the
//                workgroups of one XCD hit the same one or two blocks in its L2.
//   fallback     Larsson-Sadakane style prefix doubling on ranks for the groups still tied (only
//                pathological, highly repetitive blocks get here), using the same MSD/wave
//                machinery on 32-bit rank keys.
#include "bwt.h"
#include "prof.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

namespace bra {

#ifdef BRA_DEBUG
#define BRA_DSYNC(st)                                                                                     \
    do                                                                                                    \
    {                                                                                                     \
        hipError_t _e = hipStreamSynchronize(st);                                                         \
        if (_e != hipSuccess)                                                                             \
            fprintf(stderr, "[bra dsync] %s after the launch at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
    } while (0)
#else
#define BRA_DSYNC(st) \
    do                \
    {                 \
    } while (0)
#endif

namespace {

constexpr int      TILE         = 4096;  // elements per MSD tile (256 threads x 16)
constexpr int      TPB          = 256;
constexpr int      PER_THREAD   = TILE / TPB;
constexpr uint32_t JOB_MAX      = 256;  // elements one wave sorts in registers
constexpr int      MJ_WAVES_DEF = 4;    // waves of the largest workgroup job (2 or 4; 8 / 16 -- jobs of up to 4096 -- measured slower, removed)
constexpr uint32_t DCAP_BIG     = 64;   // MSD depth after which a big bucket goes to the fallback
constexpr uint32_t DCAP_JOB     = 512;  // refinement depth after which a tied group goes to the fallback
constexpr uint32_t RANK_KEYBYTES = 4;   // rank keys are 32-bit
constexpr uint32_t CSTRIDE    = 256 + 16;  // digit-counter copies (TileStagePN, k_hist): 16 banks apart
constexpr int      SCATTER_NC = 4;  // digit-counter copies of the MSD scatter
constexpr int      HIST_NC    = 4;  // counter copies of the MSD histogram (copy = lane & (NC - 1)), [digit][copy]; 1 / 2 / 8 / 16 measured slower
constexpr uint32_t JQ_CHUNK   = 2;  // wave jobs a wave claims with one atomic (8: equal)
// Former compile-time tuning knobs are constants now: a build that still passes one fails here
// instead of measuring the default under another label.
#if defined(JOB_MIN_WAVES) || defined(MJOB_MIN_WAVES) || defined(BRA_SCATTER_NC) || defined(BRA_TILE) || defined(HD2_REFB_BITS) || \
    defined(BRA_SCAN_MIN_WAVES) || defined(BRA_HIST_NC)
#error "removed tuning macro: these values are constants in bwt.hip"
#endif
#define MJOB_MIN_WAVES 5  // min waves per SIMD of the workgroup-job kernels (merge levels are LDS-latency bound: 4 -> 5 waves 4.37 -> 4.06 ms; 6 spills)
#define JOB_MIN_WAVES 5   // min waves per SIMD of the wave-job kernel (6 spills)

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
    uint32_t start, len, kd, buf, block, gdepth, d;  // d: depth (bytes shared) of the job's sub-buckets
};

struct Group
{
    uint32_t start, len, depth, block;
};

// Every counter that many workgroups hit with device-scope atomics sits on its own 128-byte line:
// same-line atomics serialise at the memory side (about 11 ns each), which made the per-bucket
// scan cost ~58 ns per workgroup while all counters shared one line.
struct Counters
{
    alignas(128) uint32_t n_big;         // buckets appended to the next level      } one 64-bit atomic
    uint32_t n_tiles_next;               // tiles reserved for the next level        }
    alignas(128) uint32_t n_jobs;        // wave jobs (<= JOB_MAX elements)         } one 64-bit atomic
    uint32_t n_mjobs;                    // workgroup jobs (<= mjob_max elements)   }
    alignas(128) uint32_t n_groups;      // fallback groups appended (next round)
    uint32_t g_members;                  // members of appended fallback groups
    uint32_t hmin;                       // min depth of appended fallback groups
    alignas(128) uint32_t overflow;      // a work list overflowed (fatal)
    alignas(128) uint32_t n_moved;       // elements the level's scatter moves (byte accounting)
    alignas(128) uint32_t n_elems_next;
    alignas(128) uint32_t n_melems;      // elements in workgroup jobs (byte accounting)
};

// A STRING-mode MSD tile as the hist and scatter kernels need it (built with the tile order, so a
// workgroup reaches its tile's data with one dependent load).
struct TileDesc
{
    uint32_t t;       // tile index (tile_hist / tile_off row)
    uint32_t bi;      // bucket
    uint32_t s0;      // slot of the tile's first element
    uint32_t cnt;     // elements in the tile
    uint32_t d;       // bucket depth (digit = byte d, carried in the payloads)
    uint32_t bstart;  // bucket slots [bstart, bstart + blen)
    uint32_t blen;
    uint32_t buf;     // KV buffer holding the bucket
    uint32_t poff;    // the block's packed key string (PackDesc): offset, bits, bits per character
    uint32_t nbits;
    uint32_t kd;      // the payloads carry digits [kd, kd + CARRY)
    uint32_t pdig;    // 1: the bucket stayed in place, its digits are read from the payloads (not dig[])
    uint32_t pb;
};

// Ordered tile list of a level: XCD x's part is [xseg[x], xseg[x + 1]) (workgroup w works on
// XCD w % 8's part).  desc == nullptr: natural order (tile i, RANK mode).
struct TileOrder
{
    const TileDesc* desc;
    const uint32_t* xseg;
    uint32_t        natural;  // desc is in tile order: workgroup w takes tiles w, w + grid, ...
};

// List position of a workgroup's i-th tile, or ~0u when its XCD's part is exhausted.
__device__ __forceinline__ uint32_t tile_pos(const TileOrder& o, uint32_t i, uint32_t ntiles)
{
    if (!o.desc || o.natural)
    {
        const uint32_t t = blockIdx.x + i * gridDim.x;
        return t < ntiles ? t : ~0u;
    }
    const uint32_t x = blockIdx.x & 7, l = blockIdx.x >> 3, g = gridDim.x >> 3;
    const uint32_t p = o.xseg[x] + l + i * g;
    return p < o.xseg[x + 1] ? p : ~0u;
}

// List position of wave wv's i-th tile when every wave of a workgroup takes tiles on its own (the
// workgroup's XCD part is shared by its waves as if they were 4 x as many workgroups).
__device__ __forceinline__ uint32_t tile_pos_wave(const TileOrder& o, uint32_t i, uint32_t ntiles, uint32_t wv, uint32_t wpg)
{
    if (!o.desc || o.natural)
    {
        const uint32_t t = blockIdx.x * wpg + wv + i * gridDim.x * wpg;
        return t < ntiles ? t : ~0u;
    }
    const uint32_t x = blockIdx.x & 7, l = (blockIdx.x >> 3) * wpg + wv, g = (gridDim.x >> 3) * wpg;
    const uint32_t p = o.xseg[x] + l + i * g;
    return p < o.xseg[x + 1] ? p : ~0u;
}

// -------------------------------------------------------------------------------------------------
// Packed key strings.  Rotations are sorted on their characters mapped to their ranks in the block's
// alphabet (a monotone map: the order of rotations is unchanged) and packed b bits per character,
// b = ceil(log2(alphabet size)) in 1..8.  A key byte -- a "virtual byte", the unit of every digit,
// depth and key below -- then covers 8 / b characters: synthetic text (26 letters, b = 5) needs
// 1.6x fewer MSD levels and job rounds than raw bytes, 16-symbol data (b = 4) 2x fewer, uniform
// random bytes (b = 8) are unchanged.  Block k's packed string is its n*b-bit cyclic bitstream
// (MSB first) followed by its first PACK_EXT_BITS bits again, so any window of up to 136 bits
// starting inside the stream is contiguous; it lives at packed + PackDesc.poff.  Two rotations are
// identical once they agree on nvb = ceil(n*b / 8) virtual bytes.
// -------------------------------------------------------------------------------------------------
struct PackDesc
{
    uint32_t poff;   // byte offset of the block's packed string (block offset + PACK_PAD * block)
    uint32_t nbits;  // n * b
    uint32_t b;      // bits per character
    uint32_t nvb;    // ceil(nbits / 8): depth at which tied rotations are identical
};
constexpr uint32_t PACK_PAD      = 96;   // bytes reserved per block beyond n (16-byte alignment, the extension, overreads)
constexpr uint32_t PACK_EXT_BITS = 384;  // cyclic continuation written after the stream (>= 136 bits + 16-byte overread)

typedef uint64_t __attribute__((aligned(1))) u64_unaligned;
typedef uint4 __attribute__((aligned(1))) uint4_u;

// bit position of rotation idx's virtual byte vd in its block's cyclic bitstream
__device__ __forceinline__ uint32_t pk_bitpos(uint32_t b, uint32_t nbits, uint32_t idx, uint32_t vd)
{
    uint32_t bp = idx * b + 8u * vd;
    if (bp >= nbits)
        bp %= nbits;
    return bp;
}

// 128 bits of a packed string from bit bp: w0 = bits [bp, bp + 64), w1 = the next 64 except its
// lowest bp % 8 bits (zero): one unaligned 16-byte load.  The consumers use at most the top 56
// bits of w1 (the round-2 key bits of a job), so the byte after the 16 is not loaded (that second
// load per element cost as much as the first in the job kernels' memory requests).
__device__ __forceinline__ void pk_load128(const uint8_t* __restrict__ pk, uint32_t bp, uint64_t& w0, uint64_t& w1)
{
    const uint8_t* p  = pk + (bp >> 3);
    const uint4    q  = *reinterpret_cast<const uint4_u*>(p);
    uint64_t       a  = __builtin_bswap64(((uint64_t) q.y << 32) | q.x);
    uint64_t       c  = __builtin_bswap64(((uint64_t) q.w << 32) | q.z);
    const uint32_t sh = bp & 7;
    if (sh)
    {
        a = (a << sh) | (c >> (64 - sh));
        c <<= sh;
    }
    w0 = a;
    w1 = c;
}

// 64 bits of a packed string from bit bp (bit bp in the MSB), except the lowest bp % 8 bits (zero):
// one unaligned 8-byte load.  The consumers use the top 48 (job keys) or 32 (MSD payload digits).
__device__ __forceinline__ uint64_t pk_load64(const uint8_t* __restrict__ pk, uint32_t bp)
{
    const uint8_t* p = pk + (bp >> 3);
    return __builtin_bswap64(*reinterpret_cast<const u64_unaligned*>(p)) << (bp & 7);
}

// STRING-mode payload (64 bits): the rotation index in bits 0-23, the rotation's BWT output byte
// (the input byte before it, cyclically) in bits 24-31, and CARRY digits, virtual bytes
// [kd, kd + CARRY) of the rotation, big-endian in bits 32-63.  A bucket at depth d reads digit
// d - kd; the scatter that moves an element into a bucket at depth kd + CARRY gathers the next
// CARRY digits (one 64-bit packed load), so an element costs one gather per CARRY MSD levels.
// The output byte rides along from level 0 (read there from the tile's input bytes), so the job
// that finally places the rotation needs no gather for it (5 carried digits without it cost one
// more random byte load per element in the jobs than 4 digits cost in extra MSD re-gathers).
constexpr uint32_t CARRY = 4;
__device__ __forceinline__ uint32_t p_idx(uint64_t P) { return (uint32_t) P & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t p_digit(uint64_t P, uint32_t j) { return (uint32_t) (P >> (56 - 8 * j)) & 0xFFu; }
// payload P re-carrying virtual bytes [vd, vd + CARRY) of its rotation (index and output byte kept)
__device__ __forceinline__ uint64_t p_make(const uint8_t* __restrict__ pk, uint32_t b, uint32_t nbits, uint32_t vd, uint64_t P)
{
    const uint64_t k = pk_load64(pk, pk_bitpos(b, nbits, p_idx(P), vd));
    return (k & 0xFFFFFFFF00000000ull) | (P & 0xFFFFFFFFull);
}

// Counters of one call: slot 0 holds the call-wide lists (jobs, workgroup jobs, fallback groups,
// overflow); slot k >= 1 holds what the scan of MSD level k - 1 appended for level k (n_big,
// n_tiles_next, and the byte-accounting counts).  Every slot is zeroed once, by k_ctr_init at the
// start of the call (or of a fallback round), so no kernel ever resets a counter a later kernel
// reads, and the host never has to copy a level's counts back before it launches the next level.
constexpr uint32_t MAX_LEVELS = DCAP_BIG + 2;  // slot 0 + one per STRING level (depth <= DCAP_BIG)

__global__ void k_ctr_init(Counters* ctr, uint32_t nslots)
{
    uint32_t* w = reinterpret_cast<uint32_t*>(ctr);
    for (uint32_t i = threadIdx.x; i < nslots * (uint32_t) (sizeof(Counters) / 4); i += blockDim.x)
        w[i] = 0;
    __syncthreads();
    if (threadIdx.x == 0)
        ctr[0].hmin = 0xFFFFFFFFu;
}

// A count an earlier kernel of the call accumulated with device-scope atomics.  Read with an
// agent-scope atomic load (global_load sc1: never served from a CU's L1 or the scalar cache) instead
// of a plain load, which the compiler may turn into a scalar load through the non-coherent K$.
__device__ __forceinline__ uint32_t dev_count(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Host mailbox record: a level's counts, written by k_publish into pinned host memory so the host
// can follow the level loop without a copy or a stream synchronisation.  `seq` is stored last.
struct Mail
{
    uint32_t n_big, n_tiles, overflow, n_groups, hmin, n_jobs, n_mjobs, n_melems, seq;
};

__global__ void k_publish(const Counters* __restrict__ g, const Counters* __restrict__ lv, Mail* __restrict__ mail, uint32_t seq)
{
    if (threadIdx.x != 0)
        return;
    const uint32_t v[8] = {lv ? dev_count(&lv->n_big) : 0u, lv ? dev_count(&lv->n_tiles_next) : 0u, dev_count(&g->overflow), dev_count(&g->n_groups),
                           dev_count(&g->hmin),  dev_count(&g->n_jobs),  dev_count(&g->n_mjobs), dev_count(&g->n_melems)};
    uint32_t* m = reinterpret_cast<uint32_t*>(mail);
    for (int i = 0; i < 8; ++i)
        __hip_atomic_store(m + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&mail->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// -------------------------------------------------------------------------------------------------
// level 0: byte histograms of input tiles
// -------------------------------------------------------------------------------------------------
struct L0Tile
{
    uint32_t block, start;
};

// ---- packing (see "Packed key strings") ----
// Presence mask of the byte values of every level-0 tile: tmask[8 * tile + w] bit v = value 32 w + v
// occurs.  Each thread marks its 16 bytes in a 256-byte LDS table (plain byte stores of 1: any
// order of same-address writes gives the same table; the OR-into-8-registers form cost 12 VALU per
// byte, 116 µs per 256 MiB), then 8 threads fold 32 entries each into a mask word; plain stores,
// no atomics (same-address device atomics from every tile of a block serialised this pass to half
// a millisecond).
__global__ void __launch_bounds__(TPB) k_alpha(const uint8_t* __restrict__ in, const BlockDesc* __restrict__ blocks,
                                               const L0Tile* __restrict__ tiles, uint32_t ntiles, uint32_t* __restrict__ tmask)
{
    __shared__ __attribute__((aligned(16))) uint8_t seen[256];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const L0Tile    T   = tiles[t];
        const BlockDesc B   = blocks[T.block];
        const uint32_t  cnt = min((uint32_t) TILE, B.len - T.start);
        const uint8_t*  p   = in + B.off + T.start;
        seen[threadIdx.x]   = 0;
        __syncthreads();
        if (cnt == TILE && (((uintptr_t) p) & 15) == 0)
        {
            const uint4    q    = reinterpret_cast<const uint4*>(p)[threadIdx.x];
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int i = 0; i < 16; ++i)
                seen[(w[i >> 2] >> (8 * (i & 3))) & 0xFFu] = 1;
        }
        else
            for (uint32_t i = threadIdx.x; i < cnt; i += TPB)
                seen[p[i]] = 1;
        __syncthreads();
        if (threadIdx.x < 8)
        {
            // entries 32 k .. 32 k + 31 (0 / 1 bytes) -> bits of mask word k
            const uint4* s = reinterpret_cast<const uint4*>(seen) + 2 * threadIdx.x;
            const uint4  a = s[0], b = s[1];
            const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            uint32_t       x    = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                x |= (((d[j] * 0x01020408u) >> 24) & 0xFu) << (4 * j);  // bytes 0..3 (each 0 / 1) -> bits 0..3
            tmask[8 * (size_t) t + threadIdx.x] = x;
        }
        __syncthreads();
    }
}

// One workgroup per block: the block's presence mask (OR of its tiles' masks), bits per character
// from the alphabet size, the packed string's place.
__global__ void __launch_bounds__(TPB) k_pack_desc(const BlockDesc* __restrict__ blocks, const Bucket* __restrict__ l0b, uint32_t nblocks,
                                                   const uint32_t* __restrict__ tmask, uint32_t* __restrict__ amask, PackDesc* __restrict__ pk)
{
    __shared__ uint32_t part[TPB / WAVE][8];
    for (uint32_t k = blockIdx.x; k < nblocks; k += gridDim.x)
    {
        const BlockDesc B  = blocks[k];
        const uint32_t  t0 = l0b[k].tile0, nt = div_up(B.len, TILE);
        uint32_t        m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t t = threadIdx.x; t < nt; t += TPB)
        {
            const uint4 a = reinterpret_cast<const uint4*>(tmask + 8 * (size_t) (t0 + t))[0];
            const uint4 b = reinterpret_cast<const uint4*>(tmask + 8 * (size_t) (t0 + t))[1];
            m[0] |= a.x, m[1] |= a.y, m[2] |= a.z, m[3] |= a.w, m[4] |= b.x, m[5] |= b.y, m[6] |= b.z, m[7] |= b.w;
        }
        const uint32_t wv = threadIdx.x / WAVE;
#pragma unroll
        for (int w = 0; w < 8; ++w)
        {
            const uint32_t x = wave_scan<true>(m[w], 0u, OpOr());
            if (lane_id() == WAVE - 1)
                part[wv][w] = x;
        }
        __syncthreads();
        if (threadIdx.x == 0)
        {
            uint32_t a = 0;
            for (int w = 0; w < 8; ++w)
            {
                uint32_t x = 0;
                for (uint32_t v = 0; v < TPB / WAVE; ++v)
                    x |= part[v][w];
                amask[8 * k + w] = x;
                a += __popc(x);
            }
            const uint32_t b  = (a <= 2) ? 1u : 32u - __clz(a - 1);
            const uint32_t nb = B.len * b;
            pk[k]             = PackDesc{(uint32_t) ((B.off + (uint64_t) PACK_PAD * k + 15) & ~15ull), nb, b, (nb + 7) / 8};
        }
        __syncthreads();
    }
}

// The packed strings.  Per level-0 tile: the character codes (rank of the byte value in the block's
// alphabet) are staged in LDS, every 8 consecutive characters give exactly b output bytes (8 b
// bits, MSB first), assembled in LDS and stored with 16-byte stores.  The last tile of a block also
// writes the cyclic extension (codes of the block's first characters again).
constexpr uint32_t PACK_XCH = PACK_EXT_BITS + 64;  // characters staged beyond a block's last tile (b >= 1)
__global__ void __launch_bounds__(TPB) k_pack(const uint8_t* __restrict__ in, const BlockDesc* __restrict__ blocks,
                                              const L0Tile* __restrict__ tiles, uint32_t ntiles, const uint32_t* __restrict__ amask,
                                              const PackDesc* __restrict__ pkd, uint8_t* __restrict__ packed)
{
    __shared__ uint8_t  rank[256];
    __shared__ __attribute__((aligned(16))) uint8_t code[TILE + PACK_XCH];
    __shared__ __attribute__((aligned(16))) uint8_t obuf[TILE + PACK_XCH];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const L0Tile T = tiles[t];
        {
            // rank of byte value v = number of present values below it
            const uint32_t* m = amask + 8 * T.block;
            const uint32_t  v = threadIdx.x, w = v >> 5;
            uint32_t        r = __popc(m[w] & ((1u << (v & 31)) - 1u));
            for (uint32_t k = 0; k < w; ++k)
                r += __popc(m[k]);
            rank[v] = (uint8_t) r;
        }
        __syncthreads();
        const BlockDesc B    = blocks[T.block];
        const PackDesc  P    = pkd[T.block];
        const uint8_t*  src  = in + B.off + T.start;
        const uint32_t  b    = P.b;
        const uint32_t  cnt  = min((uint32_t) TILE, B.len - T.start);
        const bool      last = T.start + TILE >= B.len;
        // characters to emit: the tile's, plus (last tile) enough of the cyclic continuation to
        // cover PACK_EXT_BITS bits, in whole groups of 8
        const uint32_t  ngrp = last ? (cnt * b + PACK_EXT_BITS + 8 * b - 1) / (8 * b) : cnt / 8;
        const uint32_t  nch  = 8 * ngrp;
        if (cnt == TILE && (((uintptr_t) src) & 15) == 0)
        {
            const uint4    q    = reinterpret_cast<const uint4*>(src)[threadIdx.x];
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
            uint32_t       o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                o[k] = (uint32_t) rank[w[k] & 0xFF] | (uint32_t) rank[(w[k] >> 8) & 0xFF] << 8 | (uint32_t) rank[(w[k] >> 16) & 0xFF] << 16 |
                       (uint32_t) rank[w[k] >> 24] << 24;
            reinterpret_cast<uint4*>(code)[threadIdx.x] = make_uint4(o[0], o[1], o[2], o[3]);
            for (uint32_t i = TILE + threadIdx.x; i < nch; i += TPB)
                code[i] = rank[in[B.off + (T.start + i) % B.len]];
        }
        else
            for (uint32_t i = threadIdx.x; i < nch; i += TPB)
            {
                uint32_t c = T.start + i;
                if (c >= B.len)
                    c %= B.len;
                code[i] = rank[in[B.off + c]];
            }
        __syncthreads();
        for (uint32_t g = threadIdx.x; g < ngrp; g += TPB)
        {
            const uint2    q   = reinterpret_cast<const uint2*>(code)[g];
            uint64_t       acc = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                acc = (acc << b) | ((i < 4 ? q.x >> (8 * i) : q.y >> (8 * (i - 4))) & 0xFFu);
            acc <<= 64 - 8 * b;  // the group's 8 b bits, MSB first
            for (uint32_t k = 0; k < b; ++k)
                obuf[g * b + k] = (uint8_t) (acc >> (56 - 8 * k));
        }
        __syncthreads();
        uint8_t*       out  = packed + P.poff + (size_t) T.start * b / 8;  // 16-byte aligned (tile starts are multiples of 4096)
        const uint32_t nout = ngrp * b;
        for (uint32_t i = threadIdx.x; i < (nout + 15) / 16; i += TPB)
            reinterpret_cast<uint4*>(out)[i] = reinterpret_cast<const uint4*>(obuf)[i];
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------------------
// level 0: histograms of the rotations' first virtual byte per tile
// -------------------------------------------------------------------------------------------------
// A level-0 tile's packed window in LDS: the bytes of its rotations' first characters plus 16 more
// (tile starts are multiples of 4096 characters, so the window starts on a 16-byte boundary of the
// packed string).  win_bits64 reads 64 bits from any bit of it.
__device__ __forceinline__ void load_window(const uint8_t* __restrict__ pk, uint32_t start, uint32_t cnt, uint32_t b, uint8_t* win)
{
    const uint4*   src = reinterpret_cast<const uint4*>(pk + (start * b) / 8);
    const uint32_t nq  = ((cnt * b + 7) / 8 + 16 + 15) / 16;
    for (uint32_t i = threadIdx.x; i < nq; i += TPB)
        reinterpret_cast<uint4*>(win)[i] = src[i];
}

__device__ __forceinline__ uint64_t win_bits64(const uint8_t* win, uint32_t bit)
{
    const uint32_t* w  = reinterpret_cast<const uint32_t*>(win) + (bit >> 5);
    const uint64_t  hi = ((uint64_t) __builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
    const uint32_t  s  = bit & 31;
    return s ? (hi << s) | (__builtin_bswap32(w[2]) >> (32 - s)) : hi;
}

__global__ void __launch_bounds__(TPB) k_l0_hist(const uint8_t* __restrict__ packed, const BlockDesc* __restrict__ blocks,
                                                 const PackDesc* __restrict__ pkd, const L0Tile* __restrict__ tiles, uint32_t ntiles,
                                                 uint32_t* __restrict__ tile_hist)
{
    __shared__ uint32_t h[SCATTER_NC * CSTRIDE];  // counter copies, see TileStagePN
    __shared__ __attribute__((aligned(16))) uint8_t win[TILE + 64];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
#pragma unroll
        for (int c = 0; c < SCATTER_NC; ++c)
            h[c * CSTRIDE + threadIdx.x] = 0;
        const L0Tile    T   = tiles[t];
        const BlockDesc B   = blocks[T.block];
        const PackDesc  P   = pkd[T.block];
        const uint32_t  cnt = min((uint32_t) TILE, B.len - T.start);
        load_window(packed + P.poff, T.start, cnt, P.b, win);
        __syncthreads();
        const uint32_t cp = (uint32_t) (lane_id() & (SCATTER_NC - 1)) * CSTRIDE;
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i)
        {
            const uint32_t e = threadIdx.x + i * TPB;
            if (e < cnt)
                atomicAdd(&h[cp + (uint32_t) (win_bits64(win, e * P.b) >> 56)], 1u);
        }
        __syncthreads();
        uint32_t tot = 0;
#pragma unroll
        for (int c = 0; c < SCATTER_NC; ++c)
            tot += h[c * CSTRIDE + threadIdx.x];
        tile_hist[(size_t) t * 256 + threadIdx.x] = tot;
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

// STRING mode: the element's payload carries the digit (byte B.d of its rotation, see p_digit);
// nothing else is read.  RANK mode: the digit
// comes from the 32-bit rank key.
template <uint32_t MODE>
__global__ void __launch_bounds__(TPB) k_hist(const Bucket* __restrict__ buckets, const uint32_t* __restrict__ tile_bucket,
                                              const uint64_t* __restrict__ key0, const uint64_t* __restrict__ key1,
                                              const uint32_t* __restrict__ pay0, const uint32_t* __restrict__ pay1,
                                              uint32_t* __restrict__ tile_hist, const Counters* __restrict__ lv, TileOrder to,
                                              const uint8_t* __restrict__ dig0, const uint8_t* __restrict__ dig1)
{
    const uint32_t ntiles = dev_count(&lv->n_tiles_next);
    __shared__ uint32_t h[256];
    if (MODE == MODE_STRING)
    {
        // One wave per tile (no workgroup barriers: most tiles past level 1 are a small bucket's only
        // tile, and the workgroup form spent its time in the two barriers and the per-tile setup).
        // STRING digits come from the byte array the previous scatter wrote beside the payloads
        // (dig[buf][slot] = the element's digit at this level): 16 contiguous digits per lane and
        // 1 KiB step, 4 steps per tile.  The next tile's descriptor is loaded before the current one
        // is counted.
        // Counters [digit][copy], HIST_NC copies, copy = lane % HIST_NC: the lanes of one atomic that
        // share a digit hit HIST_NC different banks (skewed digits: few lanes per address), and the
        // read-back of a lane's 4 digits is 4 x HIST_NC contiguous words.
        __shared__ __attribute__((aligned(16))) uint32_t hw[TPB / 64][256 * HIST_NC];
        const uint32_t      wv = wave_id(), lane = (uint32_t) lane_id();
        uint32_t* const     hc = hw[wv];
        const uint32_t      cp = lane & (HIST_NC - 1);
        uint32_t            p  = tile_pos_wave(to, 0, ntiles, wv, TPB / 64);
        TileDesc            D{};
        if (p != ~0u)
            D = to.desc[p];
        for (uint32_t it = 1; p != ~0u; ++it)
        {
            const uint32_t pn = tile_pos_wave(to, it, ntiles, wv, TPB / 64);
            TileDesc       Dn{};
            if (pn != ~0u)
                Dn = to.desc[pn];
#pragma unroll
            for (uint32_t c = 0; c < 256 * HIST_NC / 256; ++c)
                reinterpret_cast<uint4*>(hc)[c * 64 + lane] = make_uint4(0, 0, 0, 0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): without it the wave's own LDS phases overlapped (wrong counts, GPU-measured)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (D.pdig)
            {
                // digits still in the payloads (the bucket did not move at the previous level)
                const uint64_t* pay = (D.buf ? key1 : key0) + D.s0;
                const uint32_t  jj  = D.d - D.kd;
                for (uint32_t i = lane; i < D.cnt; i += 64)
                    atomicAdd(&hc[p_digit(pay[i], jj) * HIST_NC + cp], 1u);
            }
            else if (D.cnt == TILE)
            {
                // a full tile: the four 16-byte loads in flight together, no per-digit guards
                const uint8_t* g = (D.buf ? dig1 : dig0) + D.s0;
                uint4          w4[TILE / 1024];
#pragma unroll
                for (int j = 0; j < TILE / 1024; ++j)
                    w4[j] = *reinterpret_cast<const uint4_u*>(g + j * 1024 + lane * 16);
#pragma unroll
                for (int j = 0; j < TILE / 1024; ++j)
                {
                    const uint32_t wd[4] = {w4[j].x, w4[j].y, w4[j].z, w4[j].w};
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        atomicAdd(&hc[((wd[i >> 2] >> (8 * (i & 3))) & 0xFFu) * HIST_NC + cp], 1u);
                }
            }
            else
            {
                const uint8_t* g = (D.buf ? dig1 : dig0) + D.s0;
                for (uint32_t e = lane * 16; e < D.cnt; e += 1024)
                {
                    uint32_t x[4] = {0, 0, 0, 0};
                    if (e + 16 <= D.cnt)
                    {
                        const uint4 q = *reinterpret_cast<const uint4_u*>(g + e);
                        x[0] = q.x, x[1] = q.y, x[2] = q.z, x[3] = q.w;
                    }
                    else
                        for (uint32_t i = 0; e + i < D.cnt && i < 16; ++i)
                            x[i >> 2] |= (uint32_t) g[e + i] << (8 * (i & 3));
                    const uint32_t m = min(16u, D.cnt - e);
                    for (uint32_t i = 0; i < m; ++i)
                        atomicAdd(&hc[((x[i >> 2] >> (8 * (i & 3))) & 0xFFu) * HIST_NC + cp], 1u);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): without it the wave's own LDS phases overlapped (wrong counts, GPU-measured)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t tot[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
            {
                uint32_t t = 0;
                if constexpr (HIST_NC >= 4)
                {
                    const uint4* row = reinterpret_cast<const uint4*>(&hc[(lane * 4 + k) * HIST_NC]);
#pragma unroll
                    for (int c = 0; c < HIST_NC / 4; ++c)
                    {
                        const uint4 h = row[c];
                        t += h.x + h.y + h.z + h.w;
                    }
                }
                else
#pragma unroll
                    for (int c = 0; c < HIST_NC; ++c)
                        t += hc[(lane * 4 + k) * HIST_NC + c];
                tot[k] = t;
            }
            reinterpret_cast<uint4*>(tile_hist + (size_t) D.t * 256)[lane] = make_uint4(tot[0], tot[1], tot[2], tot[3]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): without it the wave's own LDS phases overlapped (wrong counts, GPU-measured)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            p = pn;
            D = Dn;
        }
        return;
    }
    for (uint32_t it = 0;; ++it)
    {
        const uint32_t p = tile_pos(to, it, ntiles);
        if (p == ~0u)
            break;
        h[threadIdx.x] = 0;
        __syncthreads();
        uint32_t t;
        if (MODE == MODE_STRING)
        {
            const TileDesc  D   = to.desc[p];
            const uint64_t* pay = (D.buf ? key1 : key0) + D.s0;
            const uint32_t  j   = D.d - D.kd;
            uint32_t        v[PER_THREAD];
#pragma unroll
            for (int i = 0; i < PER_THREAD; ++i)
            {
                const uint32_t e = threadIdx.x + i * TPB;
                v[i]             = e < D.cnt ? p_digit(pay[e], j) : 0u;
            }
#pragma unroll
            for (int i = 0; i < PER_THREAD; ++i)
                if (threadIdx.x + i * TPB < D.cnt)
                    atomicAdd(&h[v[i]], 1u);
            t = D.t;
        }
        else
        {
            t                     = p;
            const Bucket    B     = buckets[tile_bucket[t]];
            const uint32_t  first = (t - B.tile0) * TILE;
            const uint32_t  cnt   = min((uint32_t) TILE, B.len - first);
            const uint64_t* key   = (B.buf ? key1 : key0) + (size_t) B.start + first;
            for (uint32_t i = threadIdx.x; i < cnt; i += TPB)
                atomicAdd(&h[key_digit(key[i], B.d, B.kd)], 1u);
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
    const BlockDesc* blocks;
    const Bucket*   buckets;
    uint32_t        nbuckets;
    const uint32_t* tile_hist;
    uint32_t*       tile_off;
    uint8_t*        nomove;
    Bucket*         next;
    uint32_t        cap_next;
    uint32_t*       tile_bucket_next;  // tile -> bucket map of the next level
    TileDesc*       tdesc_next;        // STRING: descriptors of the next level's tiles in tile order
    uint32_t        cap_tiles;
    Job*            jobs;
    uint32_t        cap_jobs;
    Job*            mjobs;
    uint32_t        cap_mjobs;
    Group*          groups;
    uint32_t        cap_groups;
    Counters*       ctr;       // call-wide lists (slot 0)
    uint32_t        dcap;      // STRING: depth cap for big buckets
    uint32_t        account;   // keep the byte-accounting counters (profiling)
    uint32_t        mjob_max;  // largest workgroup job (256 * waves; JOB_MAX = no workgroup jobs)
    const Counters* lin;       // this level's bucket count (n_big); null: nbuckets (level 0)
    Counters*       lout;      // the next level's buckets / tiles / byte accounting
    const PackDesc* pk;        // STRING: packed key strings per block
    const uint32_t* btot;      // level 0: per-bucket digit totals (k_l0_colscan) instead of the tile rows
    uint32_t*       bbase;     // level 0: per-bucket sub-bucket starts (| NEXT_FLAG), added to the tiles' running counts by the scatter
};

// One wave per bucket (SCAN_WAVES buckets per workgroup), lane = 4 consecutive digits.  Sub-bucket offsets
// per tile; the sub-buckets become wave jobs (consecutive sub-buckets of <= JOB_MAX elements packed
// greedily, <= JOB_MAX per job), workgroup jobs (<= mjob_max), next-level buckets (with their
// tiles) or fallback groups.  The four waves' list slots are reserved with one atomic per
// list per workgroup (jobs and workgroup jobs share a 64-bit atomic, so do buckets and tiles).
constexpr int SCAN_WAVES = 4;  // buckets (waves) per scan workgroup: 16 and 8 measured slower (waves of one workgroup wait for its largest bucket)

struct ScanWaveCounts
{
    uint32_t jobs, mjobs, big, tiles, groups, moved, melems, elems_next, gmembers, hmin;
};

template <uint32_t MODE>
__global__ void __launch_bounds__(64 * SCAN_WAVES) k_scan(ScanArgs a)
{
    __shared__ uint32_t       key_s[SCAN_WAVES][256];
    __shared__ uint32_t       jlen_s[SCAN_WAVES][256];
    __shared__ uint8_t        nx_s[SCAN_WAVES][256];
    __shared__ ScanWaveCounts cnt_s[SCAN_WAVES];
    __shared__ uint32_t       base_s[SCAN_WAVES][5];  // jobs, mjobs, big, tiles, groups
    const int                 lane = lane_id(), w = (int) wave_id();
    const uint32_t            nbuckets = a.lin ? dev_count(&a.lin->n_big) : a.nbuckets;
    const uint32_t            bstride  = gridDim.x * SCAN_WAVES;
    for (uint32_t b0 = blockIdx.x * SCAN_WAVES; b0 < nbuckets; b0 += bstride)
    {
        const uint32_t bi     = b0 + w;
        const bool     active = bi < nbuckets;
        Bucket         B{};
        if (active)
            B = a.buckets[bi];
#ifdef BRA_DEBUG
        if (active && lane == 0)
        {
            const BlockDesc BD = a.blocks[B.block];
            BRA_DCHECK(B.start >= BD.off && B.start + B.len <= BD.off + BD.len, "scan bucket %u start %u len %u block %u off %llu blen %u d %u",
                       bi, B.start, B.len, B.block, (unsigned long long) BD.off, BD.len, B.d);
        }
#endif
        const uint32_t ntiles = (active && !a.btot) ? div_up(B.len, TILE) : 0;
        const uint4*   th     = reinterpret_cast<const uint4*>(a.tile_hist + (size_t) B.tile0 * 256) + lane;
        uint32_t       tot[4] = {0, 0, 0, 0};
        if (a.btot && active)
        {
            const uint4 q = reinterpret_cast<const uint4*>(a.btot + (size_t) bi * 256)[lane];
            tot[0] = q.x, tot[1] = q.y, tot[2] = q.z, tot[3] = q.w;
        }
        {
            uint32_t t = 0;
            for (; t + 8 <= ntiles; t += 8)
            {
                uint4 h[8];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    h[u] = th[(size_t) (t + u) * 64];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                {
                    tot[0] += h[u].x;
                    tot[1] += h[u].y;
                    tot[2] += h[u].z;
                    tot[3] += h[u].w;
                }
            }
            for (; t < ntiles; ++t)
            {
                const uint4 h = th[(size_t) t * 64];
                tot[0] += h.x;
                tot[1] += h.y;
                tot[2] += h.z;
                tot[3] += h.w;
            }
        }
        uint32_t base[4];
        wave_excl_sum4(tot, base);
        {
            // bit 31 (STRING mode): the sub-bucket is a next-level bucket (the scatter re-gathers its
            // payload digits when the carried ones run out; slots are < 2^31)
            uint32_t flag[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const bool nb = (MODE == MODE_STRING) && tot[r] > a.mjob_max && B.d + 1 < a.dcap;
                flag[r]       = nb ? 0x80000000u : 0u;
            }
            uint4*   to     = reinterpret_cast<uint4*>(a.tile_off + (size_t) B.tile0 * 256) + lane;
            uint32_t run[4] = {B.start + base[0], B.start + base[1], B.start + base[2], B.start + base[3]};
            if (a.bbase && active)
                reinterpret_cast<uint4*>(a.bbase + (size_t) bi * 256)[lane] =
                    make_uint4(run[0] | flag[0], run[1] | flag[1], run[2] | flag[2], run[3] | flag[3]);
            for (uint32_t t = 0; t < ntiles; ++t)
            {
                const uint4 h        = th[(size_t) t * 64];
                to[(size_t) t * 64] = make_uint4(run[0] | flag[0], run[1] | flag[1], run[2] | flag[2], run[3] | flag[3]);
                run[0] += h.x;
                run[1] += h.y;
                run[2] += h.z;
                run[3] += h.w;
            }
        }
        const bool     nomove = active && __any(tot[0] == B.len || tot[1] == B.len || tot[2] == B.len || tot[3] == B.len);
        // STRING mode: the next bucket's payloads carry digits [kd, kd + CARRY); a bucket that does
        // not move but continues needs its payloads re-gathered in place when they run out (nomove
        // code 2), otherwise it is left alone (code 1)
        const bool     regather = (MODE == MODE_STRING) && (B.buf == 2u || B.d + 1 - B.kd >= CARRY);
        const uint32_t kd       = (MODE == MODE_STRING) ? (B.buf == 2u ? 1u : (regather ? B.d + 1 : B.kd)) : eff_kd(B, MODE);
        bool nm_next = false;
        if (MODE == MODE_STRING && nomove && regather)
        {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                nm_next |= (tot[r] == B.len) && tot[r] > a.mjob_max && B.d + 1 < a.dcap;
            nm_next = __any(nm_next);
        }
        const uint32_t nd     = B.d + 1;
        const uint32_t obuf   = (B.buf == 2u) ? 0u : (nomove ? B.buf : 1u - B.buf);  // buf 2 = level-0 input
        bool big[4], med[4], fin[4], nbn[4];
        bool nm_fin = false;
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            big[r] = tot[r] > a.mjob_max;
            med[r] = tot[r] > JOB_MAX && !big[r];
            fin[r] = big[r] && ((MODE == MODE_STRING) ? nd >= a.dcap : nd >= RANK_KEYBYTES);
            nbn[r] = big[r] && !fin[r];
            nm_fin |= tot[r] == B.len && fin[r];
        }
        // STRING: a bucket that stays in place as one fallback group (code 3) has its payloads' low
        // words copied to p32 by the scatter, where the group flush reads them
        nm_fin = MODE == MODE_STRING && nomove && __any(nm_fin);
        if (active && lane == 0)
            a.nomove[bi] = nomove ? (nm_fin ? 3 : (nm_next ? 2 : 1)) : 0;
        // ---- wave jobs: greedy packing of consecutive sub-buckets of <= JOB_MAX elements ----
        // The non-empty sub-buckets form a list in digit order; a wave-job sub-bucket weighs its
        // size, a larger one JOB_MAX + 1 (it never shares a job).  A job starting at entry i takes
        // entries i .. next(i) - 1, next(i) = the first entry whose end weight exceeds the start
        // weight + JOB_MAX (binary search on the weight prefix); the jobs are the chain from entry 0
        // (one lane follows it: one step per job).  Greedy packing fills wave jobs to ~175 elements
        // on text instead of ~124 with fixed windows of JOB_MAX / 2: 29 % fewer jobs, 21 % fewer
        // network stages.
        uint32_t* const Ew = key_s[w];   // end weight of each list entry
        uint32_t* const Sw = jlen_s[w];  // first slot (bucket-relative) of each list entry
        uint32_t        li[4], wt[4], wx[4], nlist;
        {
            uint32_t ne[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                ne[r] = tot[r] ? 1u : 0u;
                wt[r] = tot[r] == 0 ? 0u : (tot[r] <= JOB_MAX ? tot[r] : JOB_MAX + 1u);
            }
            wave_excl_sum4(ne, li, &nlist);
            wave_excl_sum4(wt, wx);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (tot[r])
            {
                Ew[li[r]] = wx[r] + wt[r];
                Sw[li[r]] = base[r];
                nx_s[w][li[r]] = 0;
            }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t nxt[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            nxt[r] = li[r] + 1;
            if (tot[r] && tot[r] <= JOB_MAX)
            {
                const uint32_t lim = wx[r] + JOB_MAX;
                uint32_t       lo = li[r] + 1, hi = nlist;  // first entry in [lo, hi) with Ew > lim
                while (lo < hi)
                {
                    const uint32_t m = (lo + hi) >> 1;
                    if (Ew[m] > lim)
                        hi = m;
                    else
                        lo = m + 1;
                }
                nxt[r] = lo;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (tot[r])
                Ew[li[r]] = nxt[r];  // the end weights are no longer needed: next(i) replaces them
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0)
            for (uint32_t c = 0; c < nlist; c = Ew[c])
                nx_s[w][c] = 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        bool     jstart[4];
        uint32_t js[4], jex[4], jtot, jlen[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            jstart[r] = tot[r] && tot[r] <= JOB_MAX && nx_s[w][li[r]];
            js[r]     = jstart[r] ? 1u : 0u;
            jlen[r]   = jstart[r] ? (nxt[r] < nlist ? Sw[nxt[r]] : B.len) - base[r] : 0u;
        }
        wave_excl_sum4(js, jex, &jtot);
        uint32_t jidx[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            jidx[r] = jex[r];
        // ---- workgroup jobs, next-level buckets, fallback groups ----
        uint32_t cm[4], cb[4], ct[4], cg[4], mex[4], bex[4], tex[4], gex[4], ntl[4];
        uint32_t melems = 0, enext = 0, gmem = 0, gmin = 0xFFFFFFFFu;
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            ntl[r] = nbn[r] ? div_up(tot[r], TILE) : 0;
            cm[r]  = med[r] ? 1u : 0u;
            cb[r]  = nbn[r] ? 1u : 0u;
            ct[r]  = ntl[r];
            cg[r]  = fin[r] ? 1u : 0u;
            melems += med[r] ? tot[r] : 0;
            enext += nbn[r] ? tot[r] : 0;
            gmem += fin[r] ? tot[r] : 0;
        }
        ScanWaveCounts C{};
        wave_excl_sum4(cm, mex, &C.mjobs);
        wave_excl_sum4(cb, bex, &C.big);
        wave_excl_sum4(ct, tex, &C.tiles);
        wave_excl_sum4(cg, gex, &C.groups);
        C.jobs = active ? jtot : 0;
        if (!active)
            C.mjobs = C.big = C.tiles = C.groups = 0;
        if (a.account || C.groups)
        {
            for (int d = 32; d >= 1; d >>= 1)
            {
                melems += __shfl_xor(melems, d, WAVE);
                enext += __shfl_xor(enext, d, WAVE);
                gmem += __shfl_xor(gmem, d, WAVE);
            }
            C.melems     = active ? melems : 0;
            C.elems_next = active ? enext : 0;
            C.gmembers   = active ? gmem : 0;
            C.moved      = (active && !nomove) ? B.len : 0;
            gmin         = C.groups ? ((MODE == MODE_STRING) ? nd : B.gdepth) : 0xFFFFFFFFu;
        }
        C.hmin = gmin;
        if (lane == 0)
            cnt_s[w] = C;
        __syncthreads();
        if (threadIdx.x == 0)
        {
            uint32_t pre[5] = {0, 0, 0, 0, 0}, tj = 0, tm = 0, tb = 0, tt = 0, tg = 0;
            ScanWaveCounts T{};
            T.hmin = 0xFFFFFFFFu;
            for (int v = 0; v < SCAN_WAVES; ++v)
            {
                const ScanWaveCounts& c = cnt_s[v];
                base_s[v][0] = tj;
                base_s[v][1] = tm;
                base_s[v][2] = tb;
                base_s[v][3] = tt;
                base_s[v][4] = tg;
                tj += c.jobs;
                tm += c.mjobs;
                tb += c.big;
                tt += c.tiles;
                tg += c.groups;
                T.moved += c.moved;
                T.melems += c.melems;
                T.elems_next += c.elems_next;
                T.gmembers += c.gmembers;
                T.hmin = min(T.hmin, c.hmin);
            }
            if (tj || tm)
            {
                const unsigned long long old =
                    atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctr->n_jobs), ((unsigned long long) tm << 32) | tj);
                pre[0] = (uint32_t) old;
                pre[1] = (uint32_t) (old >> 32);
            }
            if (tb)
            {
                const unsigned long long old =
                    atomicAdd(reinterpret_cast<unsigned long long*>(&a.lout->n_big), ((unsigned long long) tt << 32) | tb);
                pre[2] = (uint32_t) old;
                pre[3] = (uint32_t) (old >> 32);
            }
            if (tg)
            {
                pre[4] = atomicAdd(&a.ctr->n_groups, tg);
                atomicAdd(&a.ctr->g_members, T.gmembers);
                atomicMin(&a.ctr->hmin, T.hmin);
            }
            if (a.account)
            {
                if (T.moved)
                    atomicAdd(&a.lout->n_moved, T.moved);
                if (T.melems)
                    atomicAdd(&a.ctr->n_melems, T.melems);
                if (T.elems_next)
                    atomicAdd(&a.lout->n_elems_next, T.elems_next);
            }
            for (int v = 0; v < SCAN_WAVES; ++v)
                for (int q = 0; q < 5; ++q)
                    base_s[v][q] += pre[q];
        }
        __syncthreads();
        if (active)
        {
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const uint32_t s0 = B.start + base[r];
                if (jstart[r])
                {
                    const uint32_t slot = base_s[w][0] + jidx[r];
                    if (slot < a.cap_jobs)
                        // STRING: the kd field of a job flags a single sub-bucket (its keys can start at
                        // the first unshared byte; jobs do not use kd otherwise)
                        a.jobs[slot] = Job{s0, jlen[r], MODE == MODE_STRING ? (nxt[r] == li[r] + 1 ? 1u : 0u) : kd, obuf, B.block, B.gdepth, nd};
                    else
                        atomicExch(&a.ctr->overflow, 1u);
                }
                if (med[r])
                {
                    const uint32_t slot = base_s[w][1] + mex[r];
                    if (slot < a.cap_mjobs)
                        a.mjobs[slot] = Job{s0, tot[r], kd, obuf, B.block, B.gdepth, nd};
                    else
                        atomicExch(&a.ctr->overflow, 1u);
                }
                if (nbn[r])
                {
                    const uint32_t slot = base_s[w][2] + bex[r], t0 = base_s[w][3] + tex[r];
                    if (slot < a.cap_next && t0 + ntl[r] <= a.cap_tiles)
                    {
                        a.next[slot] = Bucket{s0, tot[r], nd, kd, B.block, obuf, B.gdepth, t0};
                        for (uint32_t t = 0; t < ntl[r]; ++t)
                            a.tile_bucket_next[t0 + t] = slot;
                        if (MODE == MODE_STRING)
                        {
                            const PackDesc P = a.pk[B.block];
                            for (uint32_t t = 0; t < ntl[r]; ++t)
                                a.tdesc_next[t0 + t] = TileDesc{t0 + t, slot, s0 + t * TILE, min((uint32_t) TILE, tot[r] - t * TILE), nd,
                                                                s0, tot[r], obuf, P.poff, P.nbits, kd,
                                                                (nomove && !regather) ? 1u : 0u, P.b};
                        }
                    }
                    else
                        atomicExch(&a.ctr->overflow, 1u);
                }
                if (fin[r])
                {
                    const uint32_t gdep = (MODE == MODE_STRING) ? nd : B.gdepth;
                    const uint32_t slot = base_s[w][4] + gex[r];
                    if (slot < a.cap_groups)
                        a.groups[slot] = Group{s0, tot[r], gdep, B.block | (obuf << 31)};
                    else
                        atomicExch(&a.ctr->overflow, 1u);
                }
            }
        }
        __syncthreads();
    }
}

struct TileStage
{
    uint64_t key[TILE];
    uint32_t pay[TILE];
    uint32_t cnt[256];
    uint32_t base[256];
    uint32_t goff[256];
    uint32_t tmp[8];
};

// STRING-mode tile staging: 64-bit payloads (index + carried digits).  The digit counters come in
// NC copies (copy = lane & (NC - 1)) CSTRIDE words apart, so that lanes of one instruction with
// the same digit hit NC different counters in different banks (same-address LDS atomics
// serialise; skewed digits are the norm for text).
template <int NC, typename PAY = uint64_t>
struct TileStagePN
{
    PAY      pay[TILE];
    uint32_t cnt[NC * CSTRIDE];  // per copy: count, then the copy's first staging slot per digit
    uint32_t base[256];          // first staging slot per digit
    uint32_t goff[256];          // sub-bucket slot of the tile's first element per digit (bit 31: next-level bucket)
    uint32_t tmp[8];
};
using TileStageP = TileStagePN<1>;
using TileStageS = TileStagePN<SCATTER_NC>;
using TileStageL0 = TileStagePN<4, uint32_t>;  // level 0 stages 32-bit (digit << 24 | position) values  // level 0 (plus the input window: 4 copies cost one workgroup per CU)
constexpr uint32_t NEXT_FLAG = 0x80000000u;

template <int NC, typename PAY>
__device__ __forceinline__ void stage_zero(TileStagePN<NC, PAY>& S)
{
#pragma unroll
    for (int c = 0; c < NC; ++c)
        S.cnt[c * CSTRIDE + threadIdx.x] = 0;
}

// Ranks the tile's elements by digit in LDS and stages them in digit order; the caller reads
// S.pay[q] back in order (coalesced output runs per digit) and finds a staged element's digit
// offset as q - S.base[digit].
template <int NC, typename PAY, typename V>
__device__ __forceinline__ void stage_p(TileStagePN<NC, PAY>& S, const V (&v)[PER_THREAD], const uint32_t (&dgt)[PER_THREAD], uint32_t cnt)
{
    const uint32_t cp = (NC > 1) ? (uint32_t) (lane_id() & (NC - 1)) * CSTRIDE : 0u;
    uint32_t       rank[PER_THREAD];
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i)
    {
        const uint32_t e = threadIdx.x + i * TPB;
        if (e < cnt)
            rank[i] = atomicAdd(&S.cnt[cp + dgt[i]], 1u);
    }
    __syncthreads();
    uint32_t c[NC], tot = 0;
#pragma unroll
    for (int k = 0; k < NC; ++k)
    {
        c[k] = S.cnt[k * CSTRIDE + threadIdx.x];
        tot += c[k];
    }
    const uint32_t b    = block256_exclusive_sum(tot, S.tmp);
    S.base[threadIdx.x] = b;
    uint32_t run        = b;
#pragma unroll
    for (int k = 0; k < NC; ++k)
    {
        S.cnt[k * CSTRIDE + threadIdx.x] = run;
        run += c[k];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i)
    {
        const uint32_t e = threadIdx.x + i * TPB;
        if (e < cnt)
            S.pay[S.cnt[cp + dgt[i]] + rank[i]] = v[i];
    }
    __syncthreads();
}

// Writes the staged tile (already in TileStage.key/pay, count `cnt`, digit base `base`) to global.
__device__ __forceinline__ void stage_and_write(TileStage& S, const uint64_t (&k)[PER_THREAD], const uint32_t (&v)[PER_THREAD],
                                                const uint32_t (&dgt)[PER_THREAD], uint32_t cnt, uint32_t d, uint32_t kd,
                                                uint64_t* __restrict__ okey, uint32_t* __restrict__ opay, uint64_t lo, uint64_t hi)
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
            if (BRA_DCHECK(slot >= lo && slot < hi, "scatter slot %u outside [%llu, %llu) digit %u", slot, (unsigned long long) lo,
                           (unsigned long long) hi, dd))
            {
                okey[slot] = kk;
                opay[slot] = S.pay[q];
            }
        }
    }
}

// Level 0, per block: each tile's running per-digit count over the block's earlier tiles (into
// tile_off) and the block's digit totals.  The level-0 scan then reads 1 KiB per block instead of
// walking the block's tile rows twice with one wave (256 tiles of 1 MiB blocks: the round-3 scan
// took 116 us for 256 waves); the scatter adds the scan's sub-bucket starts.  Four thread groups
// take a quarter of the tiles each.
constexpr uint32_t L0CS_GROUPS = 4;
__global__ void __launch_bounds__(256 * L0CS_GROUPS) k_l0_colscan(const Bucket* __restrict__ l0b, uint32_t nblocks, const uint32_t* __restrict__ tile_hist,
                                                                  uint32_t* __restrict__ tile_off, uint32_t* __restrict__ btot)
{
    __shared__ uint32_t part[L0CS_GROUPS][256];
    const uint32_t      d = threadIdx.x & 255u, g = threadIdx.x >> 8;
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const Bucket    B   = l0b[b];
        const uint32_t  nt  = div_up(B.len, TILE);
        const uint32_t  per = div_up(nt, L0CS_GROUPS);
        const uint32_t  t0 = min(nt, g * per), t1 = min(nt, t0 + per);
        const uint32_t* th = tile_hist + (size_t) B.tile0 * 256 + d;
        uint32_t*       to = tile_off + (size_t) B.tile0 * 256 + d;
        uint32_t        sum = 0, t = t0;
        for (; t + 8 <= t1; t += 8)
        {
            uint32_t h[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                h[u] = th[(size_t) (t + u) * 256];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                sum += h[u];
        }
        for (; t < t1; ++t)
            sum += th[(size_t) t * 256];
        part[g][d] = sum;
        __syncthreads();
        uint32_t run = 0, tot = 0;
#pragma unroll
        for (uint32_t k = 0; k < L0CS_GROUPS; ++k)
        {
            const uint32_t x = part[k][d];
            run += k < g ? x : 0u;
            tot += x;
        }
        for (t = t0; t + 8 <= t1; t += 8)
        {
            uint32_t h[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                h[u] = th[(size_t) (t + u) * 256];
#pragma unroll
            for (int u = 0; u < 8; ++u)
            {
                to[(size_t) (t + u) * 256] = run;
                run += h[u];
            }
        }
        for (; t < t1; ++t)
        {
            const uint32_t h = th[(size_t) t * 256];
            to[(size_t) t * 256] = run;
            run += h;
        }
        if (g == 0)
            btot[(size_t) b * 256 + d] = tot;
        __syncthreads();
    }
}

// Level 0: every element gets its payload carrying virtual bytes 1..CARRY (the next digits) and its
// BWT output byte.
__global__ void __launch_bounds__(TPB) k_l0_scatter(const uint8_t* __restrict__ in, const uint32_t* __restrict__ amask,
                                                    const uint8_t* __restrict__ packed, const BlockDesc* __restrict__ blocks,
                                                    const PackDesc* __restrict__ pkd, const L0Tile* __restrict__ tiles, uint32_t ntiles,
                                                    const uint32_t* __restrict__ tile_off, const uint32_t* __restrict__ l0base,
                                                    uint64_t* __restrict__ opay, uint8_t* __restrict__ odig, uint32_t* __restrict__ p32)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    TileStageL0& S   = *reinterpret_cast<TileStageL0*>(smem);
    uint8_t*     win = reinterpret_cast<uint8_t*>(smem + sizeof(TileStageL0));  // TILE + 48 bytes, 16-aligned
    __shared__ uint8_t  inv_s[256];
    __shared__ uint32_t prev_s;
    // XCD-major tile order: workgroup w runs on XCD w % 8 and takes tiles from the XCD's contiguous
    // eighth of the list, so the neighbouring output runs that adjacent tiles write to one digit's
    // sub-bucket meet in the same L2 (in list order they went to eight different L2s and reached
    // HBM as partial lines)
    const bool     xm  = gridDim.x >= 8 && (gridDim.x & 7) == 0;
    const uint32_t per = xm ? div_up(ntiles, 8u) : ntiles;
    const uint32_t t0  = xm ? (blockIdx.x & 7) * per : 0u;
    const uint32_t t1  = min(ntiles, t0 + per);
    for (uint32_t t = t0 + (xm ? blockIdx.x >> 3 : blockIdx.x); t < t1; t += xm ? gridDim.x >> 3 : gridDim.x)
    {
        const L0Tile    T   = tiles[t];
        const BlockDesc B   = blocks[T.block];
        const PackDesc  P   = pkd[T.block];
        const uint32_t  cnt = min((uint32_t) TILE, B.len - T.start);
        load_window(packed + P.poff, T.start, cnt, P.b, win);
        stage_zero(S);
        S.goff[threadIdx.x] = tile_off[(size_t) t * 256 + threadIdx.x] + l0base[(size_t) T.block * 256 + threadIdx.x];  // (bit 31: next-level bucket)
        {
            // alphabet rank -> byte value (the packing's map, inverted): thread v = byte value v
            const uint32_t  vv = threadIdx.x;
            const uint32_t* m  = amask + 8 * T.block;
            uint32_t        r  = __popc(m[vv >> 5] & ((1u << (vv & 31)) - 1u));
            for (uint32_t k = 0; k < (vv >> 5); ++k)
                r += __popc(m[k]);
            if ((m[vv >> 5] >> (vv & 31)) & 1u)
                inv_s[r] = (uint8_t) vv;
            if (threadIdx.x == 0)
                prev_s = in[B.off + (T.start ? T.start - 1 : B.len - 1)];
        }
        __syncthreads();
        uint32_t v[PER_THREAD], dg[PER_THREAD];
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i)
        {
            const uint32_t e = threadIdx.x + i * TPB;
            dg[i]            = (e < cnt) ? (uint32_t) (win_bits64(win, e * P.b) >> 56) : 0u;  // virtual byte 0
            v[i]             = (dg[i] << 24) | e;
        }
        stage_p(S, v, dg, cnt);
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i)
        {
            const uint32_t q = threadIdx.x + i * TPB;
            if (q < cnt)
            {
                const uint32_t vv   = (uint32_t) S.pay[q];
                const uint32_t dd   = vv >> 24, e = vv & 0xFFFFFFu;
                const uint32_t g    = S.goff[dd];
                const uint32_t slot = (g & ~NEXT_FLAG) + (q - S.base[dd]);
                const uint64_t kk   = win_bits64(win, e * P.b);  // virtual bytes 0..7: keep bytes 1..CARRY
                const uint32_t pos  = T.start + e;
                // the output byte: the character before the element in the packed window, mapped
                // back from its alphabet rank (the tile's first element: the byte read ahead)
                const uint32_t lb = e ? inv_s[(uint32_t) (win_bits64(win, (e - 1) * P.b) >> (64 - P.b))] : prev_s;
                if (BRA_DCHECK(slot >= B.off && slot < B.off + B.len, "l0 scatter slot %u outside block %u", slot, T.block))
                {
                    if (g & NEXT_FLAG)
                    {
                        opay[slot] = ((kk << 8) & 0xFFFFFFFF00000000ull) | ((uint64_t) lb << 24) | pos;
                        odig[slot] = (uint8_t) (kk >> 48);  // virtual byte 1: the level-1 digit
                    }
                    else
                        p32[slot] = (lb << 24) | pos;  // a job's element: the job reads only the low word
                }
            }
        }
        __syncthreads();
    }
}

// STRING-mode MSD scatter of 64-bit payloads.  An element whose sub-bucket continues as a
// next-level bucket (tile_off bit 31) at depth kd + CARRY gets the next CARRY digits gathered from
// the input (the block is in the XCD's L2); all others keep their payload (jobs only use the
// index).  nomove 1: the bucket stays as it is; 2: it stays in place but continues and its
// payloads are re-gathered in place.
__global__ void __launch_bounds__(TPB, 4) k_scatter_p(const uint8_t* __restrict__ packed, const uint8_t* __restrict__ nomove,
                                                   const uint32_t* __restrict__ tile_off, uint64_t* __restrict__ pay0,
                                                   uint64_t* __restrict__ pay1, const Counters* __restrict__ lv, TileOrder to,
                                                   uint8_t* __restrict__ dig0, uint8_t* __restrict__ dig1, uint32_t* __restrict__ p32)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    TileStageS&    S      = *reinterpret_cast<TileStageS*>(smem);
    const uint32_t ntiles = dev_count(&lv->n_tiles_next);
    for (uint32_t it = 0;; ++it)
    {
        const uint32_t p = tile_pos(to, it, ntiles);
        if (p == ~0u)
            break;
        const TileDesc D  = to.desc[p];
        const uint32_t nm = nomove[D.bi];
        if (nm == 1)
            continue;  // uniform per workgroup: the bucket stays as it is (the next level reads its digits from the payloads)
        if (nm == 3)
        {
            // the bucket stays where it is as one fallback group: its payloads' low words to p32
            const uint64_t* ip = (D.buf ? pay1 : pay0) + D.s0;
            for (uint32_t e = threadIdx.x; e < D.cnt; e += TPB)
                p32[D.s0 + e] = (uint32_t) ip[e];
            continue;
        }
        const uint32_t t   = D.t;
        const uint8_t* pk  = packed + D.poff;
        const uint32_t cnt = D.cnt;
        struct
        {
            uint32_t start, len, d, buf;
        } B{D.bstart, D.blen, D.d, D.buf};
        const uint32_t  j  = B.d - D.kd;              // this level's digit in the payload
        const bool      rg = j + 1 >= CARRY;          // next-level buckets start a new carry
        const uint32_t  dn = B.d + 1;                 // their first digit's depth
        const size_t    s0 = D.s0;
        uint64_t*       ip = (B.buf ? pay1 : pay0) + s0;
        uint8_t*        id = (B.buf ? dig1 : dig0) + s0;
        if (nm == 2)
        {
            uint64_t v[PER_THREAD];
#pragma unroll
            for (int i = 0; i < PER_THREAD; ++i)
            {
                const uint32_t e = threadIdx.x + i * TPB;
                if (e < cnt)
                    v[i] = ip[e];
            }
#pragma unroll
            for (int i = 0; i < PER_THREAD; ++i)
            {
                const uint32_t e = threadIdx.x + i * TPB;
                if (e < cnt)
                {
                    const uint64_t np = p_make(pk, D.pb, D.nbits, dn, v[i]);
                    ip[e]             = np;
                    id[e]             = (uint8_t) p_digit(np, 0);
                }
            }
            continue;
        }
        uint64_t* op        = B.buf ? pay0 : pay1;
        uint8_t*  od        = B.buf ? dig0 : dig1;
        stage_zero(S);
        S.goff[threadIdx.x] = tile_off[(size_t) t * 256 + threadIdx.x];
        __syncthreads();
        uint64_t v[PER_THREAD];
        uint32_t dg[PER_THREAD];
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i)
        {
            const uint32_t e = threadIdx.x + i * TPB;
            v[i]             = (e < cnt) ? ip[e] : 0ull;
            dg[i]            = p_digit(v[i], j);
        }
        stage_p(S, v, dg, cnt);
        // slot and (re-gathered) payload of each staged element, stored at once (keeping all 16
        // in registers until a separate store loop cost 2x the VGPRs: 2 waves per SIMD)
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i)
        {
            const uint32_t q = threadIdx.x + i * TPB;
            if (q < cnt)
            {
                const uint64_t vv   = S.pay[q];
                const uint32_t dd   = p_digit(vv, j), g = S.goff[dd];
                const uint32_t slot = (g & ~NEXT_FLAG) + (q - S.base[dd]);
                uint64_t       nv   = vv;
                if (rg && (g & NEXT_FLAG))
                {
                    nv = p_make(pk, D.pb, D.nbits, dn, vv);
                }
                if (BRA_DCHECK(slot >= B.start && slot < B.start + B.len, "scatter slot %u outside [%u, +%u)", slot, B.start, B.len))
                {
                    if (g & NEXT_FLAG)
                    {
                        op[slot] = nv;
                        od[slot] = (uint8_t) (rg ? p_digit(nv, 0) : p_digit(vv, j + 1));  // the next level's digit, for its histogram
                    }
                    else
                        p32[slot] = (uint32_t) vv;  // a job's or fallback group's element: only the low word is read again
                }
            }
        }
        __syncthreads();
    }
}

// RANK-mode MSD scatter (fallback rounds): 8-byte keys + payloads.
__global__ void __launch_bounds__(TPB) k_scatter(const Bucket* __restrict__ buckets, const uint8_t* __restrict__ nomove,
                                                 const uint32_t* __restrict__ tile_bucket, const Counters* __restrict__ lv,
                                                 const uint32_t* __restrict__ tile_off, uint64_t* __restrict__ key0,
                                                 uint64_t* __restrict__ key1, uint32_t* __restrict__ pay0, uint32_t* __restrict__ pay1,
                                                 uint32_t mode)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    TileStage&     S      = *reinterpret_cast<TileStage*>(smem);
    const uint32_t ntiles = dev_count(&lv->n_tiles_next);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x)
    {
        const uint32_t bi = tile_bucket[t];
        if (nomove[bi])
            continue;  // uniform per workgroup
        const Bucket    B     = buckets[bi];
        const uint32_t  first = (t - B.tile0) * TILE;
        uint32_t        cnt   = min((uint32_t) TILE, B.len - first);
        if (!BRA_DCHECK(t >= B.tile0 && first < B.len && B.buf < 2, "scatter tile %u bucket %u tile0 %u len %u buf %u", t, bi, B.tile0, B.len, B.buf))
            cnt = 0;
        const uint32_t  kd    = (mode == MODE_STRING && B.d - B.kd >= 8) ? B.d : B.kd;
        const uint64_t* ik    = B.buf ? key1 : key0;
        const uint32_t* ip    = B.buf ? pay1 : pay0;
        uint64_t*       ok    = B.buf ? key0 : key1;
        uint32_t*       op    = B.buf ? pay0 : pay1;
        S.cnt[threadIdx.x]    = 0;
        S.goff[threadIdx.x]   = tile_off[(size_t) t * 256 + threadIdx.x] & ~NEXT_FLAG;
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
        stage_and_write(S, k, v, dg, cnt, B.d, kd, ok, op, B.start, (uint64_t) B.start + B.len);
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------------------
// jobs: <= 256*W elements sorted by W waves (4 per lane; W = 1 wave jobs, W > 1 workgroup jobs).
// STRING mode sorts by 128-bit keys: the group id in the top GBITS bits, then the next
// 128 - GBITS bits of the rotation gathered from the input at the group's depth (15 bytes per round
// for W = 1, 14 for W > 1).  Round 1's groups are the job's sub-buckets (their digit at depth d-1);
// every later round only handles the elements still tied, compacted with a job-wide prefix count
// and re-sorted with a network of the compacted size.  A round's active elements occupy an
// increasing list of job positions; the sort permutes elements over that list.  STRING mode stops
// when nothing is tied, when the depth reaches n (ties = identical rotations) or at the depth cap
// (the tied groups go to the fallback).  RANK mode sorts once by the 32-bit rank key and emits
// the equal-key groups as the next fallback round's groups.
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
    uint32_t         hstep;    // RANK mode: depth added to a subgroup (min depth of the round)
    uint32_t         xcd_major;  // jobs ordered by job_order(): XCD x works on jobs [xseg[x], xseg[x+1])
    uint32_t         xseg[9];
    const uint32_t*  dxseg;    // non-null: the per-XCD list ranges live in device memory (k_job_prefix), not in xseg
    uint32_t*        jq;       // dynamic order (xcd_major only): per-XCD claim counters, 32 dwords apart; null = static ranges
    uint32_t         jq_chunk; // jobs a wave claims at once
    const uint8_t*   packed;   // STRING: packed key strings (keys are gathered from them)
    const PackDesc*  pk;
    const uint32_t*  p32;      // STRING: the job elements' payload low words (BWT byte << 24 | rotation), by slot
};

// Hardware id (0-7) of the XCD the calling wave runs on.  Speed only: the job queues below stay
// correct whatever it returns, since every wave drains all eight queues before it exits.
__device__ __forceinline__ uint32_t xcc_id()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x & 7u;
}

// Dynamic job order: the waves of XCD x claim chunks of XCD x's part of the block-major list with
// an atomic counter, so all waves of an XCD work on the same one or two blocks at any time (the
// static stride let late-starting workgroups begin at the head of the list while early ones were
// at its tail, spreading an XCD's gathers over all its blocks).  A wave whose own part is
// exhausted helps the other XCDs' parts, so the launch drains every job whatever the placement.
// Returns the first job of the claimed chunk and its end, or false when all parts are drained.
struct JobClaim
{
    uint32_t x0, t;
};

// Called by a whole wave (wave-uniform control flow; lane 0 performs the atomic).
__device__ __forceinline__ bool job_claim(const JobArgs& a, const uint32_t* xs, JobClaim& c, uint32_t chunk, uint32_t& first, uint32_t& end)
{
    while (c.t < 8)
    {
        const uint32_t x = (c.x0 + c.t) & 7u, lo = xs[x], hi = xs[x + 1];
        uint32_t       b = 0;
        if (lane_id() == 0)
            b = atomicAdd(&a.jq[x * 32], chunk);
        b = __builtin_amdgcn_readfirstlane(b);
        if (b < hi - lo)
        {
            first = lo + b;
            end   = min(hi, first + chunk);
            return true;
        }
        ++c.t;
    }
    return false;
}

// The per-XCD list ranges into LDS (from device memory when k_job_prefix computed them, else from
// the kernel arguments); every thread of the workgroup calls it.
__device__ __forceinline__ void load_xseg(const JobArgs& a, uint32_t* xs)
{
    if (threadIdx.x < 9)
        xs[threadIdx.x] = a.dxseg ? dev_count(a.dxseg + threadIdx.x) : a.xseg[threadIdx.x];
    __syncthreads();
}

// Job index ranges per workgroup.  With xcd_major, workgroup w runs on XCD w % 8 (the dispatcher's
// round-robin; only speed depends on it) and walks that XCD's list, where the jobs of the blocks
// b = x (mod 8) are stored in block order: the workgroups of one XCD then gather from the same one
// or two blocks at a time, which stay resident in that XCD's 4 MiB L2.
struct JobRange
{
    uint32_t first, end, step;
};

__device__ __forceinline__ JobRange job_range(const JobArgs& a, const uint32_t* xs, uint32_t unit, uint32_t units_per_wg)
{
    if (a.xcd_major)
    {
        const uint32_t x = blockIdx.x & 7, l = blockIdx.x >> 3, g = gridDim.x >> 3;
        return JobRange{xs[x] + l * units_per_wg + unit, xs[x + 1], g * units_per_wg};
    }
    return JobRange{blockIdx.x * units_per_wg + unit, a.njobs, gridDim.x * units_per_wg};
}

template <int W>
struct JobGeom
{
    static constexpr int      LOGS  = (W == 1) ? 8 : (W == 2) ? 9 : (W == 4) ? 10 : (W == 8) ? 11 : 12;  // log2(256 * W)
    static constexpr int      GBITS = LOGS;                                // group id bits (top of the key)
    static constexpr uint64_t SMASK = (1ull << LOGS) - 1;                  // slot bits (bottom of the key)
    // 64-bit keys: group id | the rotation's next packed bits | slot.  Round 1 (no group bits)
    // carries 6-7 rotation bytes, later rounds 5-6.  A 64-bit compare-exchange is 7 VALU against
    // the 10 / 13 of the 96 / 128-bit keys of round 2, and the keys take half the registers; the
    // elements still tied after round 1 (about a quarter of them on text) take another round.
    static constexpr int      KD    = 2;
    static constexpr uint32_t KBITS = 32 * KD;
    static constexpr uint32_t ADV   = (KBITS - GBITS - LOGS) / 8;          // whole rotation bytes per key
    static constexpr uint32_t ADV1  = (KBITS - LOGS) / 8;                  // round 1: no group bits
};

template <int W>
struct JobLds
{
    static constexpr int KD = JobGeom<W>::KD;
#ifdef BRA_JOB_AUDIT
    static constexpr int KH = 256 * W;  // the audit keeps a sort's output here
#else
    // Wave jobs use kh only for the small sorts (<= 128 keys) and as 32-bit compaction scratch, so
    // 1 KiB instead of 2: 4.6 KiB per wave fits 8 four-wave workgroups per CU (8 waves per SIMD)
    // where 5.6 KiB fitted 7.  (Measured equal, round 6: 1.744 / 1.746 vs 1.749 / 1.740 ms -- the
    // seventh wave already hides what occupancy can.)
    static constexpr int KH = (W == 1) ? 128 : 256 * W;
#endif
    uint64_t kh[KH];        // neighbour keys, merge levels, small sorts; as uint32_t: compaction scratch
    uint64_t wx[256 * W];   // STRING: the 64 rotation bits after each element's round-1 key (the round-2 key bits)
    uint32_t v[256 * W];    // payload of every slot of the current round (the keys carry the slot)
    uint32_t nx[W];         // group-end scratch (the first head of each wave)
    uint16_t pos[256 * W];  // job position of each active slot (increasing)
    uint32_t agg[W];        // per-wave aggregates: the group-start max-scan (and the audit)
    uint32_t aggf[W];       // per-wave "any slot tied" flags, exchanged with agg
    uint32_t agg2[W];       // per-wave tied counts (job_excl_count)
    uint32_t aggm[W];       // per-wave group-end min-scan aggregates (job_group_ends)
};

template <int W>
__device__ __forceinline__ void job_sync()
{
    if (W > 1)
        __syncthreads();
    else
    {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}


template <int W>
__device__ __forceinline__ bool job_any(bool x)
{
    if (W > 1)
        return __syncthreads_or(x);
    return __any(x);
}



// Inclusive max-scan of x over the job's slots and whether any lane of the job has `any` set, with
// one barrier for W > 1: the wave aggregates and flags go through their own LDS words, which are
// written again only in the next round's scan -- every wave has passed the tied-count exchange or
// the compaction barriers (or left the job) by then, so no second barrier guards their reuse.
template <int W>
__device__ __forceinline__ bool job_max_scan_any(uint32_t (&x)[4], bool any, JobLds<W>& S, int wj)
{
    wave_max_scan4(x);
    const bool wany = __builtin_amdgcn_ballot_w64(any) != 0;
    if (W == 1)
        return wany;
    if (lane_id() == 63)
        S.agg[wj] = x[3];
    if (lane_id() == 0)
        S.aggf[wj] = wany ? 1u : 0u;
    job_sync<W>();
    uint32_t ex = 0, f = 0;
#pragma unroll
    for (int w = 0; w < W; ++w)
    {
        if (w < wj)
            ex = max(ex, S.agg[w]);
        f |= S.aggf[w];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
        x[r] = max(x[r], ex);
    return __builtin_amdgcn_readfirstlane(f) != 0;
}


template <int W>
__device__ __forceinline__ void job_min_rscan(uint32_t (&x)[4], JobLds<W>& S, int wj)
{
    wave_min_rscan4(x);
    if (W > 1)
    {
        if (lane_id() == 0)
            S.aggm[wj] = x[0];
        job_sync<W>();
        uint32_t ex = 0xFFFFFFFFu;
        for (int w = wj + 1; w < W; ++w)
            ex = min(ex, S.aggm[w]);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            x[r] = min(x[r], ex);
        job_sync<W>();
    }
}


template <int W>
__device__ __forceinline__ void job_excl_count(const bool (&f)[4], uint32_t (&ex)[4], uint32_t& total, JobLds<W>& S, int wj)
{
    const int lane = lane_id();
    uint32_t  c    = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        ex[r] = c;
        c += f[r] ? 1u : 0u;
    }
    const uint32_t x    = wave_scan<true>(c, 0u, OpAdd());
    uint32_t       wtot = __builtin_amdgcn_readlane(x, 63), pre = x - c;
    if (W > 1)
    {
        // (agg2 is written again only in the next round's count, after the compaction barriers:
        // no second barrier)
        if (lane == 63)
            S.agg2[wj] = x;
        job_sync<W>();
        uint32_t before = 0, all = 0;
        for (int w = 0; w < W; ++w)
        {
            const uint32_t a = S.agg2[w];
            if (w < wj)
                before += a;
            all += a;
        }
        pre += before;
        wtot = all;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
        ex[r] += pre;
    total = wtot;
}

// One bitonic stage whose partners sit LM lanes away (same element r): exchanged with DPP /
// permlane swaps.  k[i][r] = dword i of element r's key.
// Keys of KD dwords (2: 64 bits, the job sorts; 3 / 4: 96 / 128 bits).
template <int KD>
__device__ __forceinline__ void cxk(uint32_t (&k)[KD][4], int r, const uint32_t (&o)[KD], uint64_t keep_min)
{
    if constexpr (KD == 2)
        cx64(k[0][r], k[1][r], o[0], o[1], keep_min);
    else if constexpr (KD == 3)
        cx96(k[0][r], k[1][r], k[2][r], o[0], o[1], o[2], keep_min);
    else
        cx128(k[0][r], k[1][r], k[2][r], k[3][r], o[0], o[1], o[2], o[3], keep_min);
}

template <int KD>
__device__ __forceinline__ void cxk_pair(uint32_t (&a)[KD], uint32_t (&b)[KD], uint64_t asc)
{
    if constexpr (KD == 2)
        cx64_pair(a[0], a[1], b[0], b[1], asc);
    else if constexpr (KD == 3)
        cx96_pair(a[0], a[1], a[2], b[0], b[1], b[2], asc);
    else
        cx128_pair(a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3], asc);
}

template <int LM, int KD>
__device__ __forceinline__ void net_stage_lanes(uint32_t (&k)[KD][4], uint64_t keep_min)
{
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        uint32_t o[KD];
#pragma unroll
        for (int i = 0; i < KD; ++i)
            o[i] = xlane<LM>(k[i][r]);
        cxk<KD>(k, r, o, keep_min);
    }
}

// Stage whose partners sit 16 or 32 lanes away (J = 64 or 128 slots): a permlane swap of the
// registers of elements (0, 1) and of (2, 3) gathers each partner pair into ONE lane (element r0's
// pair in the lower rows, r1's in the upper rows, the lower slot in the first register), an
// in-lane compare-exchange orders it, and the same swap puts the elements back: 7.5 VALU per
// element instead of 18 with per-dword partner fetches.
// Rows of x and y exchanged as the permlane swap does (LM 16: x's odd rows <-> y's even rows; 32: x's
// upper half <-> y's lower half).
template <int LM>
__device__ __forceinline__ void swap_rows(uint32_t& x, uint32_t& y)
{
    const auto t = (LM == 16) ? __builtin_amdgcn_permlane16_swap(x, y, false, false) : __builtin_amdgcn_permlane32_swap(x, y, false, false);
    x = t[0];
    y = t[1];
}

template <int LM, int KD>
__device__ __forceinline__ void net_stage_swap(uint32_t (&k)[KD][4], uint64_t asc)
{
#pragma unroll
    for (int q = 0; q < 4; q += 2)
    {
        uint32_t a[KD], b[KD];
#pragma unroll
        for (int i = 0; i < KD; ++i)
        {
            a[i] = k[i][q];
            b[i] = k[i][q + 1];
            swap_rows<LM>(a[i], b[i]);
        }
        cxk_pair<KD>(a, b, asc);
#pragma unroll
        for (int i = 0; i < KD; ++i)
        {
            swap_rows<LM>(a[i], b[i]);
            k[i][q]     = a[i];
            k[i][q + 1] = b[i];
        }
    }
}

// Stage (SIZE, J) of the bitonic network and, recursively, the rest of its merge phase.  All
// stage parameters are compile-time, so a phase is straight-line code with the keys in fixed
// registers (a runtime stage loop made the compiler copy every key between register sets at each
// stage join).
// Lane masks of the network as compile-time constants (a ballot of a lane predicate reached the
// inline-asm compare-exchanges only after a copy through a VGPR: 2 VALU per stage).  Slot e of lane
// l is 4 l + r (+ a wave-uniform multiple of 256, eb): bit l of lanes_where<X, Y>() is set iff
// ((4 l) & X) == 0 equals ((4 l) & Y) == 0 (Y = 0: iff ((4 l) & X) == 0).
template <uint32_t X, uint32_t Y>
constexpr uint64_t lanes_where()
{
    uint64_t m = 0;
    for (uint32_t l = 0; l < 64; ++l)
    {
        const bool a = ((4 * l) & X) == 0, b = Y ? ((4 * l) & Y) == 0 : true;
        if (a == b)
            m |= 1ull << l;
    }
    return m;
}

// Lanes that keep the minimum at stage (SIZE, J >= 4) / sort ascending in phase SIZE.
template <int SIZE, int J>
__device__ __forceinline__ uint64_t net_keep_min(uint32_t eb)
{
    if constexpr (SIZE < 256)
        return lanes_where<SIZE, J>();
    else
        return (eb & SIZE) == 0 ? lanes_where<J, 0>() : ~lanes_where<J, 0>();
}
template <int SIZE>
__device__ __forceinline__ uint64_t net_asc(uint32_t eb)
{
    if constexpr (SIZE < 4)
        return ~0ull;  // in-lane phase 2: direction from r (see net_stage)
    else if constexpr (SIZE < 256)
        return lanes_where<SIZE, 0>();
    else
        return (eb & SIZE) == 0 ? ~0ull : 0ull;
}

template <int W, int KD, int SIZE, int J>
__device__ __forceinline__ void net_stage(uint32_t (&k)[KD][4], JobLds<W>& S, uint32_t e0)
{
    static_assert(J < 256, "cross-wave merges are merge_level's");
    const uint32_t eb = __builtin_amdgcn_readfirstlane(e0) & ~255u;  // the wave's slot base (lane 0: 4 * 0)
    if constexpr (J == 64 || J == 128)
        net_stage_swap<J / 4, KD>(k, net_asc<SIZE>(eb));
    else if constexpr (J >= 4)
        net_stage_lanes<J / 4, KD>(k, net_keep_min<SIZE, J>(eb));
    else
    {
        // partners in the same lane: r and r ^ J; ascending where (slot & SIZE) == 0
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const int q = r ^ J;
            if (q > r)
            {
                const uint64_t asc = SIZE == 2 ? ((r & 2) == 0 ? ~0ull : 0ull) : net_asc<SIZE>(eb);
                uint32_t a[KD], b[KD];
#pragma unroll
                for (int i = 0; i < KD; ++i)
                {
                    a[i] = k[i][r];
                    b[i] = k[i][q];
                }
                cxk_pair<KD>(a, b, asc);
#pragma unroll
                for (int i = 0; i < KD; ++i)
                {
                    k[i][r] = a[i];
                    k[i][q] = b[i];
                }
            }
        }
    }
    if constexpr (J > 1)
        net_stage<W, KD, SIZE, J / 2>(k, S, e0);
}

template <int W, int KD, int SIZE>
__device__ __forceinline__ void net_phase(uint32_t (&k)[KD][4], JobLds<W>& S, uint32_t e0)
{
    net_stage<W, KD, SIZE, SIZE / 2>(k, S, e0);
}

// One merge level of a workgroup job's sort: sorted runs of m slots (in LDS) merged pairwise into
// runs of 2m.  Merge path: the lane owning output slots [e0, e0 + 4) finds how many of them come
// from the left run with one binary search (co-rank), then merges its 4 outputs sequentially
// (instead of log2(2m) compare-exchange stages, the cross-wave ones through LDS with two barriers
// each).  Equal keys (padding) take the left run first.
template <int W>
__device__ __forceinline__ void merge_level(uint32_t (&k)[2][4], JobLds<W>& S, uint32_t e0, uint32_t m)
{
    uint64_t* X = S.kh;
    job_sync<W>();
#pragma unroll
    for (int r = 0; r < 4; ++r)
        X[e0 + r] = ((uint64_t) k[1][r] << 32) | k[0][r];
    job_sync<W>();
    const uint32_t  base = e0 & ~(2 * m - 1), kk = e0 - base;
    const uint64_t* A    = X + base;
    const uint64_t* B    = X + base + m;
    // a pair whose right run is all padding (it starts with the padding key; then so is the left
    // run if it does too) is already merged: it stays as it is
    if (B[0] != ~0ull)
    {
        uint32_t lo = kk > m ? kk - m : 0u, hi = kk < m ? kk : m;  // i = outputs [0, kk) taken from A
        while (lo < hi)
        {
            const uint32_t mid = (lo + hi) >> 1;
            if (A[mid] <= B[kk - 1 - mid])
                lo = mid + 1;
            else
                hi = mid;
        }
        uint32_t i = lo, j = kk - lo;
        uint64_t a = A[min(i, m - 1)], b = B[min(j, m - 1)];
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const bool     ta = i < m && (j >= m || a <= b);
            const uint64_t o  = ta ? a : b;
            k[0][r]           = (uint32_t) o;
            k[1][r]           = (uint32_t) (o >> 32);
            if (r < 3)
            {
                if (ta)
                    a = A[min(++i, m - 1)];
                else
                    b = B[min(++j, m - 1)];
            }
        }
    }
}

// Small sorts (16 <= P <= 128 slots: the later rounds' tied elements, small jobs).  In the 4-per-lane
// layout a stage costs 4 registers' compare-exchanges whatever P is; here the keys of slots < P move
// through LDS to R = 1 (P <= 64) or 2 (P = 128) registers per lane, slot s = R * lane + r, so a
// stage costs R.  Network cost (VALU per lane): P = 16 70 + ~25 for the moves against 154, P = 64
// 147 against 390, P = 128 329 against 552 (below 16 slots the moves cost more than they save).
template <int R, uint32_t X, uint32_t Y>
constexpr uint64_t lanes_where_r()
{
    uint64_t m = 0;
    for (uint32_t l = 0; l < 64; ++l)
    {
        const bool a = ((R * l) & X) == 0, b = Y ? ((R * l) & Y) == 0 : true;
        if (a == b)
            m |= 1ull << l;
    }
    return m;
}

template <int R, int SIZE, int J>
__device__ __forceinline__ void snet_stage(uint32_t (&k)[2][4])
{
    if constexpr (J >= R)
    {
        // partner J / R lanes away; the lower slot keeps the minimum where (slot & SIZE) == 0
        constexpr uint64_t keep_min = lanes_where_r<R, SIZE, J>();
#pragma unroll
        for (int r = 0; r < R; ++r)
        {
            const uint32_t o[2] = {xlane<J / R>(k[0][r]), xlane<J / R>(k[1][r])};
            cxk<2>(k, r, o, keep_min);
        }
    }
    else
    {
        // R = 2, J = 1: the lane's own two slots, ascending where (2 lane & SIZE) == 0
        uint32_t a[2] = {k[0][0], k[1][0]}, b[2] = {k[0][1], k[1][1]};
        cxk_pair<2>(a, b, lanes_where_r<R, SIZE, 0>());
        k[0][0] = a[0];
        k[1][0] = a[1];
        k[0][1] = b[0];
        k[1][1] = b[1];
    }
    if constexpr (J > 1)
        snet_stage<R, SIZE, J / 2>(k);
}

template <int R>
__device__ __forceinline__ void snet_sort(uint32_t (&k)[2][4], int P)
{
    for (int size = 2; size <= P; size <<= 1)
        switch (size)
        {
        case 2: snet_stage<R, 2, 1>(k); break;
        case 4: snet_stage<R, 4, 2>(k); break;
        case 8: snet_stage<R, 8, 4>(k); break;
        case 16: snet_stage<R, 16, 8>(k); break;
        case 32: snet_stage<R, 32, 16>(k); break;
        case 64: snet_stage<R, 64, 32>(k); break;
        default:
            if constexpr (R == 2)
                snet_stage<R, 128, 64>(k);
            break;
        }
}

// One wave's small sort.  S.kh is free during a sort (its last readers precede the caller's barrier).
template <int W>
__device__ __forceinline__ void job_sort_small(uint32_t (&k)[2][4], int P, JobLds<W>& S)
{
    const uint32_t lane = (uint32_t) lane_id();
    uint64_t*      X    = S.kh;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (lane * 4 + r < (uint32_t) P)
            X[lane * 4 + r] = ((uint64_t) k[1][r] << 32) | k[0][r];
    job_sync<1>();
    uint32_t q[2][4];
    if (P <= 64)
    {
        const uint64_t x = lane < (uint32_t) P ? X[lane] : ~0ull;
        q[0][0]          = (uint32_t) x;
        q[1][0]          = (uint32_t) (x >> 32);
        snet_sort<1>(q, P);
        job_sync<1>();
        if (lane < (uint32_t) P)
            X[lane] = ((uint64_t) q[1][0] << 32) | q[0][0];
    }
    else
    {
#pragma unroll
        for (int r = 0; r < 2; ++r)
        {
            const uint64_t x = X[2 * lane + r];
            q[0][r]          = (uint32_t) x;
            q[1][r]          = (uint32_t) (x >> 32);
        }
        snet_sort<2>(q, P);
        job_sync<1>();
#pragma unroll
        for (int r = 0; r < 2; ++r)
            X[2 * lane + r] = ((uint64_t) q[1][r] << 32) | q[0][r];
    }
    job_sync<1>();
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (lane * 4 + r < (uint32_t) P)
        {
            const uint64_t x = X[lane * 4 + r];
            k[0][r]          = (uint32_t) x;
            k[1][r]          = (uint32_t) (x >> 32);
        }
}

// Sort of the job's 256*W 64-bit keys (4 consecutive per lane, slot e = wj*256 + lane*4 + r) over
// the first P (power of two) slots: each wave's 256 slots by the in-wave bitonic phases (DPP /
// permlane partners), then (W > 1, P > 256) merge-path levels across the waves.  Keys are unique
// (the slot is in the low bits).  The network runs on dwords (no 64-bit register pairs to keep
// together).
#ifdef BRA_JOB_AUDIT
__device__ uint32_t g_sort_fail;           // job sorts whose output was not strictly ascending (padding aside)
__device__ uint32_t g_sort_owner = ~0u;     // workgroup that dumped the first one
__device__ uint64_t g_sort_dump[2][1024];   // its input and output keys (slot order)
__device__ uint32_t g_sort_meta[4];         // W, P, the wave's xcc, the sort's index in its job
__device__ uint64_t g_sort_phase[10][1024];  // the failing sort re-run: keys after each phase
#endif

template <int W>
__device__ __forceinline__ void job_sort(uint64_t (&key)[4], int P, JobLds<W>& S, int wj)
{
    const int      lane = lane_id();
    const uint32_t e0   = wj * 256 + lane * 4;
#ifdef BRA_JOB_AUDIT
    const uint64_t kin[4] = {key[0], key[1], key[2], key[3]};
#endif
    uint32_t       k[2][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        k[0][r] = (uint32_t) key[r];
        k[1][r] = (uint32_t) (key[r] >> 32);
    }
    // A wave whose slots all hold padding keys (all ones) skips the phases that stay inside the
    // wave (SIZE <= 256: no barriers, no data from other waves); any order of equal keys is
    // sorted.  Only workgroup jobs have such waves (the tail of a job whose length is not a power
    // of two, or the waves beyond P in later rounds).
    bool dead = false;
    if (W > 1)
        dead = __builtin_amdgcn_ballot_w64((k[0][0] & k[1][0] & k[0][1] & k[1][1] & k[0][2] & k[1][2] & k[0][3] & k[1][3]) != ~0u) == 0;
    // the in-wave phases sort each wave's slots ascending (directions from the wave-local slot)
    const uint32_t el = (W > 1 && P > 256) ? (uint32_t) lane * 4 : e0;
    // Workgroup jobs (their wave 0; the other waves hold padding only): up to 64 slots -- the
    // 128-slot form raised the 4-wave kernel to 88 allocated VGPRs (a wave per SIMD less, 6 %
    // slower); up to 64 it stays at 80 (mjobs 3.20 vs 3.23 ms).
    const bool small = P >= 16 && P <= (W == 1 ? 128 : 64);
    if (small && wj == 0)
        job_sort_small<W>(k, P, S);
    for (int size = 2; !small && size <= P; size <<= 1)
    {
        if (dead && size <= 256)
            continue;
        if constexpr (W > 1)
            if (size > 256)
            {
                merge_level<W>(k, S, e0, (uint32_t) size / 2);
                continue;
            }
        switch (size)
        {
        case 2: net_phase<W, 2, 2>(k, S, el); break;
        case 4: net_phase<W, 2, 4>(k, S, el); break;
        case 8: net_phase<W, 2, 8>(k, S, el); break;
        case 16: net_phase<W, 2, 16>(k, S, el); break;
        case 32: net_phase<W, 2, 32>(k, S, el); break;
        case 64: net_phase<W, 2, 64>(k, S, el); break;
        case 128: net_phase<W, 2, 128>(k, S, el); break;
        default: net_phase<W, 2, 256>(k, S, el); break;
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
        key[r] = ((uint64_t) k[1][r] << 32) | k[0][r];
    job_sync<W>();
#ifdef BRA_JOB_AUDIT
    {
        // strictly ascending real keys over the first P slots (real keys carry their slot: unique)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            S.kh[e0 + r] = key[r];
        job_sync<W>();
        bool bad = false;
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c = e0 + r;
            if (c + 1 < (uint32_t) P && key[r] != ~0ull && !(S.kh[c + 1] > key[r]))
                bad = true;
        }
        bad = job_any<W>(bad);
        if (bad)
        {
            if (threadIdx.x == 0)
            {
                atomicAdd(&g_sort_fail, 1u);
                S.agg[0] = atomicCAS(&g_sort_owner, ~0u, blockIdx.x) == ~0u ? 1u : 0u;
            }
            job_sync<W>();
            if (S.agg[0])
            {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                {
                    g_sort_dump[0][e0 + r] = kin[r];
                    g_sort_dump[1][e0 + r] = key[r];
                }
                // the same sort again from kin, with the keys after every phase
                uint32_t kk[2][4];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                {
                    kk[0][r] = (uint32_t) kin[r];
                    kk[1][r] = (uint32_t) (kin[r] >> 32);
                }
                int ph = 0;
                for (int size = 2; size <= P; size <<= 1, ++ph)
                {
                    if (!(dead && size <= 256))
                    {
                        if constexpr (W > 1)
                            if (size > 256)
                                merge_level<W>(kk, S, e0, (uint32_t) size / 2);
                        if (size <= 256)
                            switch (size)
                            {
                            case 2: net_phase<W, 2, 2>(kk, S, el); break;
                            case 4: net_phase<W, 2, 4>(kk, S, el); break;
                            case 8: net_phase<W, 2, 8>(kk, S, el); break;
                            case 16: net_phase<W, 2, 16>(kk, S, el); break;
                            case 32: net_phase<W, 2, 32>(kk, S, el); break;
                            case 64: net_phase<W, 2, 64>(kk, S, el); break;
                            case 128: net_phase<W, 2, 128>(kk, S, el); break;
                            default: net_phase<W, 2, 256>(kk, S, el); break;
                            }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        g_sort_phase[ph][e0 + r] = ((uint64_t) kk[1][r] << 32) | kk[0][r];
                }
                if (threadIdx.x == 0)
                {
                    g_sort_meta[0] = W;
                    g_sort_meta[1] = (uint32_t) P;
                    g_sort_meta[2] = xcc_id();
                }
            }
        }
        job_sync<W>();
    }
#endif
}

// Group heads, group starts (g: max-scan of the head positions) and ties over the T active slots
// (a slot is tied when a neighbour holds the same key); km = the keys without the slot bits.
// Returns whether any slot is tied (job-wide).
template <int W>
__device__ __forceinline__ bool job_groups(const uint64_t (&km)[4], uint32_t T, JobLds<W>& S, int wj, uint32_t (&g)[4], bool (&tied)[4],
                                           bool (&hd)[4])
{
    const int lane = lane_id();
    // neighbour keys: the lane's own elements, the previous / next lane's (ds_bpermute), or (the
    // first / last lane of a wave of a workgroup job) the neighbouring wave's through LDS
    uint64_t pm = (uint64_t) __shfl_up((long long) km[3], 1, WAVE);
    uint64_t nm = (uint64_t) __shfl_down((long long) km[0], 1, WAVE);
    if (W > 1)
    {
        if (lane == 63)
            S.kh[wj * 256 + 255] = km[3];
        if (lane == 0)
            S.kh[wj * 256] = km[0];
        job_sync<W>();
        if (lane == 0 && wj > 0)
            pm = S.kh[wj * 256 - 1];
        if (lane == 63 && wj + 1 < W)
            nm = S.kh[(wj + 1) * 256];
    }
    bool any = false;
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        const uint32_t c  = wj * 256 + lane * 4 + r;
        const uint64_t qp = r ? km[r - 1] : pm;
        const uint64_t qn = r < 3 ? km[r + 1] : nm;
        hd[r]             = (c == 0) || c >= T || qp != km[r];
        g[r]              = hd[r] ? c : 0;
        tied[r]           = c < T && (!hd[r] || (c + 1 < T && qn == km[r]));
        any |= tied[r];
    }
    return job_max_scan_any<W>(g, any, S, wj);  // (its barrier also orders the S.kh reads above before later writes)
}

// Group ends (the next head after each slot, or T): only where groups are emitted (RANK mode, or
// STRING groups sent to the fallback).
template <int W>
__device__ __forceinline__ void job_group_ends(const bool (&hd)[4], uint32_t T, JobLds<W>& S, int wj, uint32_t (&gend)[4])
{
    constexpr uint32_t SLOTS = 256 * W;
    const int          lane  = lane_id();
    uint32_t           x[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
        x[r] = hd[r] ? wj * 256 + lane * 4 + r : 0xFFFFFFFFu;
    job_min_rscan<W>(x, S, wj);
    uint32_t nx3 = (uint32_t) __shfl_down((int) x[0], 1, WAVE);
    if (lane == 63)
        nx3 = 0xFFFFFFFFu;
    if (W > 1)
    {
        if (lane == 0)
            S.nx[wj] = x[0];
        job_sync<W>();
        if (lane == 63 && wj + 1 < W)
            nx3 = S.nx[wj + 1];
        job_sync<W>();
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        const uint32_t c  = wj * 256 + lane * 4 + r;
        const uint32_t nh = (c + 1 < SLOTS) ? (r < 3 ? x[r + 1] : nx3) : 0xFFFFFFFFu;
        gend[r]           = min(nh == 0xFFFFFFFFu ? SLOTS : nh, T);
    }
}

// round-1 key: the rotation's packed bits from the key's first depth, low LOGS bits = slot
template <int W>
__device__ __forceinline__ uint64_t make_key1(uint32_t slot, uint64_t w0)
{
    return (w0 & ~JobGeom<W>::SMASK) | slot;
}

// key = group | the rotation's bits (w0) shifted right by GBITS, low LOGS bits = slot
template <int W>
__device__ __forceinline__ uint64_t make_key(uint32_t grp, uint32_t slot, uint64_t w0)
{
    using G = JobGeom<W>;
    return ((((uint64_t) grp << (64 - G::GBITS)) | (w0 >> G::GBITS)) & ~G::SMASK) | slot;
}

#ifdef BRA_JOB_TIMING
// Diagnostic build only (make EXTRA=-DBRA_JOB_TIMING): shader cycles of the job phases, summed over
// the jobs by the first wave of each job, [wave jobs, workgroup jobs] x {claim + descriptor, gathers
// of round 1, sort of round 1, groups + outputs, compaction + gathers of later rounds, sorts of later
// rounds, rounds, jobs}; printed to stderr after each STRING encode.
// Accumulated per wave in LDS and added to the device totals once, when the wave leaves the kernel
// (per-phase device atomics queued behind each other and slowed the job kernels 20x).
__device__ unsigned long long g_jt[2][32];  // [10 + lg P]: round-1 sorts by log2 P, [21 + lg P]: later sorts
__device__ __forceinline__ unsigned long long* jt_slots()
{
    __shared__ unsigned long long jt_s[16][32];
    return jt_s[threadIdx.x >> 6];
}
#define JT_NOW() (wj == 0 ? (unsigned long long) clock64() : 0ull)
#define JT_ADD(i, x)                               \
    do                                             \
    {                                              \
        if (wj == 0 && lane_id() == 0)             \
            jt_slots()[i] += (unsigned long long) (x); \
    } while (0)
#define JT_INIT()                                  \
    do                                             \
    {                                              \
        if (lane_id() < 32)                        \
            jt_slots()[lane_id()] = 0;             \
    } while (0)
#define JT_FLUSH(w2)                               \
    do                                             \
    {                                              \
        if (lane_id() < 32)                        \
            atomicAdd(&g_jt[w2][lane_id()], jt_slots()[lane_id()]); \
    } while (0)
#else
#define JT_NOW() 0ull
#define JT_ADD(i, x) \
    do               \
    {                \
    } while (0)
#define JT_INIT() \
    do            \
    {             \
    } while (0)
#define JT_FLUSH(w2) \
    do               \
    {                \
    } while (0)
#endif

// Round-1 data of a STRING job's slots: v = BWT output byte << 24 | rotation, w0 / w1 = the 128
// packed bits from the job's first key byte.  (Gathering them one job ahead, with the payloads two
// jobs ahead, removed the wait before the first sort but needed 128 VGPRs, 4 waves per SIMD, and
// moved the wait to the next job's start -- behind the previous job's output stores, since the
// vector memory counter retires in issue order: no faster.)
struct JobPre
{
    uint32_t v[4];
    uint64_t w0[4], w1[4];
};

__device__ __forceinline__ PackDesc job_pack(const JobArgs& a, uint32_t MODE, uint32_t block)
{
    return MODE == MODE_STRING ? a.pk[block] : PackDesc{0, 8, 8, 1};
}

// Issue the round-1 gathers of a STRING job from its payload words (rotation in the low 24 bits).
template <int W>
__device__ __forceinline__ void job_gather1(const JobArgs& a, const Job& J, const BlockDesc& BD, const PackDesc& PK, const uint32_t (&pay)[4],
                                            int wj, JobPre& p)
{
    const uint8_t* pkb    = a.packed + PK.poff;
    const bool     single = W > 1 || J.kd == 1u;  // one shared sub-bucket: the key starts at byte d
    const uint32_t vd     = single ? J.d : J.d - 1;
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        const uint32_t c = wj * 256 + lane_id() * 4 + r;
        p.v[r]           = 0;
        p.w0[r] = p.w1[r] = 0;
        if (c < J.len)
        {
            uint32_t v = pay[r];  // output byte << 24 | rotation (the payload's low word)
            if (!BRA_DCHECK((v & 0xFFFFFFu) < BD.len, "job payload idx %u >= n %u (buf %u slot %u)", v & 0xFFFFFFu, BD.len, J.buf, J.start + c))
                v = 0;
            pk_load128(pkb, pk_bitpos(PK.b, PK.nbits, v & 0xFFFFFFu, vd), p.w0[r], p.w1[r]);
            p.v[r] = v;
        }
    }
}

template <uint32_t MODE, int W>
__device__ __forceinline__ void job_run(const JobArgs& a, const Job& J, const BlockDesc& BD, const PackDesc& PK, JobLds<W>& S, int wj)
{
    using G                 = JobGeom<W>;
    const int       lane    = lane_id();
    const uint8_t*  pkb     = a.packed + PK.poff;
    const uint64_t* K       = J.buf ? a.key1 : a.key0;
    const uint32_t* V       = J.buf ? a.pay1 : a.pay0;
    const uint32_t  boff    = (uint32_t) BD.off;
    uint64_t        key[4];  // sorted keys; after a sort: without the slot bits
    uint32_t        v[4];
    uint32_t        pos[4];  // job position of slot c
    uint32_t        g[4], gend[4];
    bool            tied[4], hd[4];
    uint32_t        T     = J.len;
    uint32_t        depth = (MODE == MODE_STRING) ? J.d : J.gdepth;
    const bool      single = MODE == MODE_STRING && (W > 1 || J.kd == 1u);
    if (!BRA_DCHECK(T <= 256u * W && J.start >= BD.off && J.start + T <= BD.off + BD.len, "job mode %u W %d start %u len %u block %u off %llu blen %u",
                    MODE, W, J.start, T, J.block, (unsigned long long) BD.off, BD.len))
        T = 0;
    [[maybe_unused]] unsigned long long jt = JT_NOW();
    JT_ADD(7, 1);
    // Round 1.  STRING: all elements share their first d-1 bytes (one parent bucket), so the key
    // is the rotation's bits from depth d-1 -- its first byte orders the packed sub-buckets, no
    // group id and no carried key needed.  The same 16-byte gather brings the next 64 bits, the
    // key bits of round 2 (S.wx): most tied elements need no second gather.  STRING payloads are
    // the 64-bit MSD payloads in the key buffers (rotation in the low bits; the top byte, an MSD
    // digit, is replaced by the rotation's BWT output byte).  RANK: the 32-bit rank key.
    JobPre gl;
    if (MODE == MODE_STRING)
    {
        uint32_t pay[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c = wj * 256 + lane * 4 + r;
            pay[r]           = c < T ? a.p32[J.start + c] : 0u;
        }
        job_gather1<W>(a, J, BD, PK, pay, wj, gl);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        const uint32_t c = wj * 256 + lane * 4 + r;
        pos[r]           = c;
        v[r]             = 0;
        key[r]           = ~0ull;  // padding: sorts last
        uint64_t wx      = 0;
        if (c < T)
        {
            if (MODE == MODE_RANK)
            {
                v[r] = V[J.start + c];  // BWT output byte << 24 | rotation
                if (!BRA_DCHECK((v[r] & 0xFFFFFFu) < BD.len, "job payload idx %u >= n %u (rank slot %u)", v[r] & 0xFFFFFFu, BD.len, J.start + c))
                    v[r] = 0;
                key[r] = K[J.start + c] | c;  // rank key in the top 32 bits
            }
            else
            {
                key[r] = make_key1<W>(c, gl.w0[r]);
                wx     = (gl.w0[r] << (8 * G::ADV1)) | (gl.w1[r] >> (64 - 8 * G::ADV1));
                v[r]   = gl.v[r];
            }
        }
        S.v[c] = v[r];
        if (MODE == MODE_STRING)
            S.wx[c] = wx;
    }
    int P = 4;
    while ((uint32_t) P < T)
        P <<= 1;
#ifdef BRA_JOB_TIMING
    if (W == 1)  // the gathers' data arrive at the sort (workgroup jobs: at its first barrier)
        __builtin_amdgcn_s_waitcnt(0);
#endif
    {
        [[maybe_unused]] const unsigned long long t1 = JT_NOW();
        JT_ADD(1, t1 - jt);
        jt = t1;
    }
    JT_ADD(10 + __builtin_ctz((unsigned) P), 1);
    job_sort<W>(key, P, S, wj);
    {
        // payloads and round-2 key bits into sorted order
        uint64_t t[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t sl = (uint32_t) (key[r] & G::SMASK);
            v[r]              = S.v[sl];
            t[r]              = MODE == MODE_STRING ? S.wx[sl] : 0ull;
            key[r] &= ~G::SMASK;
        }
        if (MODE == MODE_STRING)
        {
            job_sync<W>();
#pragma unroll
            for (int r = 0; r < 4; ++r)
                S.wx[wj * 256 + lane * 4 + r] = t[r];
        }
    }
    {
        [[maybe_unused]] const unsigned long long t1 = JT_NOW();
        JT_ADD(2, t1 - jt);
        JT_ADD(6, 1);
        jt = t1;
    }
    if (MODE == MODE_STRING)
        depth += single ? G::ADV1 : G::ADV1 - 1;
    for (uint32_t round = 1;; ++round)
    {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            S.pos[wj * 256 + lane * 4 + r] = (uint16_t) pos[r];
        const bool any    = job_groups<W>(key, T, S, wj, g, tied, hd);
        bool       finish = (MODE == MODE_RANK) || !any;
        bool final_ties = false, to_fallback = false;
        if (!finish && depth >= PK.nvb)  // tied on every bit of the cyclic string: identical rotations
            finish = final_ties = true;
        else if (!finish && depth >= a.dcap)
            finish = to_fallback = true;
        if (MODE == MODE_RANK || to_fallback)  // job-uniform
            job_group_ends<W>(hd, T, S, wj, gend);
        // ---- not finished: compact the tied slots and start the next round's key loads BEFORE
        // this round's output stores (vector-memory counts complete in issue order: a load issued
        // after a store waits for the store too) ----
        // (the keys are not needed past job_groups: key[] receives the next round's rotation bits)
        uint32_t T2 = 0;
        if (!finish)
        {
            uint32_t cx[4];
            job_excl_count<W>(tied, cx, T2, S, wj);
            if (round == 1)
            {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    key[r] = tied[r] ? S.wx[wj * 256 + lane * 4 + r] : 0ull;
            }
            // (moving the reads above before the count and leaving this barrier to the count's own,
            // W > 1, measured equal: 3.162 / 3.177 vs 3.160 / 3.161 ms)
            job_sync<W>();
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (tied[r])
                {
                    const uint32_t c = wj * 256 + lane * 4 + r;
                    S.v[cx[r]]       = v[r];
                    reinterpret_cast<uint32_t*>(S.kh)[cx[r]] = ((cx[r] - (c - g[r])) << 16) | pos[r];  // new group head | position
                    if (round == 1)
                        S.wx[cx[r]] = key[r];
                }
            job_sync<W>();
#pragma unroll
            for (int r = 0; r < 4; ++r)
            {
                const uint32_t c = wj * 256 + lane * 4 + r;
                key[r]           = 0;
                if (c < T2)
                    key[r] = round == 1 ? S.wx[c] : pk_load64(pkb, pk_bitpos(PK.b, PK.nbits, S.v[c] & 0xFFFFFFu, depth));
            }
        }
        // ---- outputs of the resolved slots (all slots when finishing) ----
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c = wj * 256 + lane * 4 + r;
            if (c >= T || (!finish && tied[r]))
                continue;
            const uint32_t slot = J.start + pos[r];
            const uint32_t idx  = v[r] & 0xFFFFFFu;
            a.fsa[slot]         = idx;
            a.L[slot]           = (uint8_t) (v[r] >> 24);
            if (MODE == MODE_RANK)
                a.isa[BD.off + idx] = J.start + S.pos[g[r]] - boff;  // block-local start of the group
            if (idx == 0)
            {
                if (MODE == MODE_RANK || final_ties)
                    a.pi[J.block] = J.start + S.pos[g[r]] - boff;
                else if (!(to_fallback && tied[r]))
                    a.pi[J.block] = slot - boff;
            }
            const bool emit = tied[r] && (MODE == MODE_RANK || to_fallback);
            if (emit && g[r] == c)
            {
                const uint32_t gl    = gend[r] - c;
                const uint32_t gd    = (MODE == MODE_RANK) ? J.gdepth + a.hstep : depth;
                const uint32_t slot2 = atomicAdd(&a.ctr->n_groups, 1u);
                if (slot2 < a.cap_groups)
                {
                    a.groups[slot2] = Group{slot, gl, gd, J.block | (1u << 30)};  // bit 30: members already in fsa
                    atomicAdd(&a.ctr->g_members, gl);
                    atomicMin(&a.ctr->hmin, gd);
                }
                else
                    atomicExch(&a.ctr->overflow, 1u);
            }
        }
        {
            [[maybe_unused]] const unsigned long long t1 = JT_NOW();
            JT_ADD(3, t1 - jt);
            jt = t1;
        }
        if (finish)
            break;
        // ---- next round on the next ADV bytes ----
        T = T2;
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c = wj * 256 + lane * 4 + r;
            pos[r]           = c;
            if (c < T)
            {
                const uint32_t gp = reinterpret_cast<const uint32_t*>(S.kh)[c];
                pos[r]            = (uint32_t) (gp & 0xFFFF);
                key[r]            = make_key<W>((uint32_t) (gp >> 16), c, key[r]);
            }
            else
                key[r] = ~0ull;
        }
        job_sync<W>();
        P = 4;
        while ((uint32_t) P < T)
            P <<= 1;
#ifdef BRA_JOB_TIMING
        if (W == 1)
            __builtin_amdgcn_s_waitcnt(0);
#endif
        {
            [[maybe_unused]] const unsigned long long t1 = JT_NOW();
            JT_ADD(4, t1 - jt);
            jt = t1;
        }
        JT_ADD(21 + __builtin_ctz((unsigned) P), 1);
        job_sort<W>(key, P, S, wj);
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            v[r] = S.v[(uint32_t) (key[r] & G::SMASK)];
            key[r] &= ~G::SMASK;
        }
        {
            [[maybe_unused]] const unsigned long long t1 = JT_NOW();
            JT_ADD(5, t1 - jt);
            JT_ADD(6, 1);
            jt = t1;
        }
        depth += G::ADV;
    }
}

template <uint32_t MODE>
__global__ void __launch_bounds__(256, JOB_MIN_WAVES) k_jobs(JobArgs a)
{
    __shared__ JobLds<1> lds[4];
    __shared__ uint32_t  xs[9];
    load_xseg(a, xs);
    const int      wl  = (int) wave_id();
    const bool     dyn = a.xcd_major && a.jq;
    const JobRange R   = job_range(a, xs, wl, 4);
    JobClaim       c{xcc_id(), 0};
    uint32_t       end = 0;
    // one call site of job_run, in a plain while loop (other loop shapes raised the register
    // allocation of the inlined job by up to 2x)
    const auto next = [&](uint32_t j) -> uint32_t {
        if (!dyn)
            return j + R.step < R.end ? j + R.step : ~0u;
        if (j + 1 < end)
            return j + 1;
        uint32_t first = 0;
        return job_claim(a, xs, c, a.jq_chunk, first, end) ? first : ~0u;
    };
    uint32_t j = dyn ? next(~0u) : (R.first < R.end ? R.first : ~0u);
    {
        [[maybe_unused]] constexpr int W = 1, wj = 0;
        JT_INIT();
        [[maybe_unused]] unsigned long long tp = JT_NOW();
        while (j != ~0u)
        {
            const Job J = a.jobs[j];
            {
                [[maybe_unused]] const unsigned long long t1 = JT_NOW();
                JT_ADD(8, t1 - tp);
            }
            job_run<MODE, 1>(a, J, a.blocks[J.block], job_pack(a, MODE, J.block), lds[wl], 0);
            tp = JT_NOW();
            j  = next(j);
        }
        if (MODE == MODE_STRING)
            JT_FLUSH(0);
    }
}

template <uint32_t MODE, int W>
__global__ void __launch_bounds__(64 * W, MJOB_MIN_WAVES) k_mjobs(JobArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    JobLds<W>&     S   = *reinterpret_cast<JobLds<W>*>(smem);
    uint32_t*      claim = reinterpret_cast<uint32_t*>(smem + sizeof(JobLds<W>));  // 2 own LDS words (launch adds 16 bytes)
    __shared__ uint32_t xs[9];
    load_xseg(a, xs);
    const bool     dyn   = a.xcd_major && a.jq;
    const JobRange R     = job_range(a, xs, 0, 1);
    JobClaim       c{xcc_id(), 0};
    uint32_t       k = 0;
    // Dynamic order: wave 0 claims the next job into claim[k & 1] and one barrier publishes it (the
    // two slots alternate, so a slot is rewritten only after every wave passed the next barrier).
    const auto next = [&](uint32_t j) -> uint32_t {
        if (!dyn)
        {
            __syncthreads();  // the LDS of the finished job is reused
            return j + R.step < R.end ? j + R.step : ~0u;
        }
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) == 0)  // wave 0
        {
            uint32_t first = 0, end = 0;
            const bool ok = job_claim(a, xs, c, 1, first, end);
            if (lane_id() == 0)
                claim[k & 1] = ok ? first : ~0u;
        }
        __syncthreads();
        return __builtin_amdgcn_readfirstlane(claim[(k++) & 1]);
    };
    const int wj = (int) wave_id();
    JT_INIT();
    [[maybe_unused]] unsigned long long tc = JT_NOW();
    uint32_t j = dyn ? next(0) : (R.first < R.end ? R.first : ~0u);
    while (j != ~0u)
    {
        {
            [[maybe_unused]] const unsigned long long t1 = JT_NOW();
            JT_ADD(0, t1 - tc);
        }
        const Job J = a.jobs[j];
        job_run<MODE, W>(a, J, a.blocks[J.block], job_pack(a, MODE, J.block), S, wj);
        tc = JT_NOW();
        j = next(j);
    }
    if (wj == 0)
        JT_FLUSH(1);
}

// ---- diagnostics: the job sort (network + merge levels) alone, on random keys ----
// Every workgroup sorts `iters` random key sets of T in [1, 256 W] elements (the job kernels' key
// layout: rotation bits above LOGS slot bits, padding all ones, a small key range so that keys
// share their high bits as tied rotations do) and checks that the T real slots come out ascending
// and as a permutation.  err[0] counts failing sorts.
__device__ __forceinline__ uint32_t sn_hash(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <int W>
__global__ void __launch_bounds__(64 * W, MJOB_MIN_WAVES) k_sortnet_test(uint32_t seed, uint32_t iters, uint32_t* __restrict__ err,
                                                                        const uint64_t* __restrict__ kfix, uint32_t tfix)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    JobLds<W>&     S    = *reinterpret_cast<JobLds<W>*>(smem);
    using G             = JobGeom<W>;
    const int      wj   = threadIdx.x >> 6, lane = lane_id();
    uint32_t       bad  = 0;
    for (uint32_t it = 0; it < iters; ++it)
    {
        const uint32_t h  = sn_hash(seed ^ (blockIdx.x * 7919u) ^ (it * 104729u));
        const uint32_t T  = kfix ? tfix : 1 + h % (256u * W);
        const uint32_t hb = 1u + (h >> 20) % 40u;  // key bits above the slot that vary
        int            P  = 4;
        while ((uint32_t) P < T)
            P <<= 1;
        uint64_t key[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c = wj * 256 + lane * 4 + r;
            const uint64_t x = ((uint64_t) sn_hash(h + 2 * c + 1) << 32 | sn_hash(h ^ (3 * c + 7))) & ((1ull << hb) - 1);
            key[r]           = kfix ? kfix[c] : c < T ? ((x << (64 - hb)) & ~G::SMASK) | c : ~0ull;
            S.v[c]           = 0;
        }
        job_sort<W>(key, P, S, wj);
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c = wj * 256 + lane * 4 + r;
            S.wx[c]          = key[r];  // (wx: kh holds fewer slots in wave jobs)
            if (c < T)
                atomicAdd(&S.v[(uint32_t) (key[r] & G::SMASK) & (256u * W - 1)], 1u);
        }
        __syncthreads();
        uint32_t b = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t c = wj * 256 + lane * 4 + r;
            if (c < T)
                b |= (S.v[c] != 1u) || (c + 1 < T && S.wx[c] >= S.wx[c + 1]) || (c + 1 == T && T < 256u * W && S.wx[c + 1] != ~0ull);
        }
        bad += __syncthreads_or(b) ? 1u : 0u;
    }
    if (threadIdx.x == 0 && bad)
        atomicAdd(err, bad);
}

// ---- job audit (diagnostics: bra_gpu_debug_rerun_jobs, and after every encode in -DBRA_JOB_AUDIT
// builds): every job's slots are counted (a slot two jobs cover is a race between them) and every
// job's output rotations are checked against its input payloads (sum and xor of the rotation
// indices); violations are printed, at most 32 per call. ----
__device__ uint32_t g_audit_prints;
__device__ uint32_t g_audit_fail;
__global__ void k_audit_cover(const Job* __restrict__ jobs, const uint32_t* __restrict__ pn, uint32_t* __restrict__ cnt)
{
    const uint32_t n = dev_count(pn);
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x)
    {
        const Job J = jobs[j];
        for (uint32_t c = threadIdx.x; c < J.len; c += blockDim.x)
            atomicAdd(&cnt[J.start + c], 1u);
    }
}
__global__ void k_audit_check(const Job* __restrict__ jobs, const uint32_t* __restrict__ pn, uint32_t kind, const uint32_t* __restrict__ p32,
                              const uint32_t* __restrict__ fsa, const uint32_t* __restrict__ cnt, const BlockDesc* __restrict__ blocks)
{
    __shared__ uint32_t s_in, s_out, x_in, x_out, over;
    const uint32_t n = dev_count(pn);
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x)
    {
        if (threadIdx.x == 0)
            s_in = s_out = x_in = x_out = over = 0;
        __syncthreads();
        const Job J = jobs[j];
        for (uint32_t c = threadIdx.x; c < J.len; c += blockDim.x)
        {
            const uint32_t a = p32[J.start + c] & 0xFFFFFFu, b = fsa[J.start + c];
            atomicAdd(&s_in, a);
            atomicAdd(&s_out, b);
            atomicXor(&x_in, a);
            atomicXor(&x_out, b);
            if (cnt[J.start + c] != 1u)
                atomicAdd(&over, 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0 && (s_in != s_out || x_in != x_out || over))
        {
            atomicAdd(&g_audit_fail, 1u);
            const uint32_t p = atomicAdd(&g_audit_prints, 1u);
            if (p < 32)
                printf("[bwt audit] %s job %u block %u (off %llu): start %u len %u kd %u buf %u d %u gdepth %u: in sum/xor %u/%u out %u/%u, %u slots shared\n",
                       kind ? "wg" : "wave", j, J.block, (unsigned long long) blocks[J.block].off, J.start, J.len, J.kd, J.buf, J.d, J.gdepth, s_in,
                       x_in, s_out, x_out, over);
        }
        __syncthreads();
    }
}

// Re-runs with another input order: the payloads of every job are put in ascending rotation order
// and then permuted by the ranks of h(seed ^ start * 2654435761, i) (ties by i), so the host can
// rebuild the exact order a failing job saw.  One workgroup (1024 threads) per job.
__device__ __forceinline__ uint32_t au_hash(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__global__ void __launch_bounds__(1024) k_audit_shuffle(const Job* __restrict__ jobs, const uint32_t* __restrict__ pn, uint32_t* __restrict__ p32,
                                                        uint32_t seed)
{
    __shared__ uint32_t pl[1024];
    __shared__ uint32_t hk[1024];
    const uint32_t n = dev_count(pn);
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x)
    {
        const Job J   = jobs[j];
        uint32_t* K   = p32;
        const uint32_t len = min(J.len, 1024u), t = threadIdx.x;
        if (t < len)
        {
            pl[t] = K[J.start + t];
            hk[t] = au_hash(seed ^ (J.start * 2654435761u) ^ au_hash(t + 1));
        }
        __syncthreads();
        uint32_t dst = 0;
        if (t < len)
        {
            // canonical rank of element t (ascending rotation index), then the slot the permutation gives that rank
            uint32_t cr = 0;
            const uint32_t me = (uint32_t) pl[t] & 0xFFFFFFu;
            for (uint32_t i = 0; i < len; ++i)
                cr += ((uint32_t) pl[i] & 0xFFFFFFu) < me;
            const uint32_t hc = hk[cr];
            for (uint32_t i = 0; i < len; ++i)
                dst += hk[i] < hc || (hk[i] == hc && i < cr);
        }
        const uint32_t mine = t < len ? pl[t] : 0;
        __syncthreads();
        if (t < len)
            K[J.start + dst] = mine;
        __syncthreads();
    }
}

// Workgroup-job size classes: a job of (256, 512] elements runs on 2 waves, (512, 1024] on 4 (never
// more waves than the job's network needs).
constexpr uint32_t MJ_CLASSES = 2;
__device__ __forceinline__ uint32_t mjob_class(uint32_t len, uint32_t classes)
{
    const uint32_t lg = 32u - (uint32_t) __builtin_clz(max(len, 257u) - 1u);  // ceil(log2(len)) >= 9
    return min(lg - 9u, classes - 1u);
}

// Block-major, XCD-major job order: key(b) = (b % 8) * kb + b / 8, size class first (classes = 1:
// one class).  With many blocks, q consecutive blocks of one XCD share a key (q = 1 up to 4096
// blocks), so the keys of a list fit the LDS counters of the ordering kernels.
__device__ __forceinline__ uint32_t job_key(const Job& J, uint32_t kb, uint32_t q, uint32_t classes)
{
    const uint32_t sc = classes > 1 ? mjob_class(J.len, classes) : 0u;
    return sc * 8 * kb + (J.block & 7u) * kb + (J.block >> 3) / q;
}

constexpr uint32_t JOB_CHUNK = 4096;  // jobs per workgroup of the ordering kernels (256 threads x 16)

// Per-key job counts.  Each workgroup counts a chunk of the list in LDS and adds its nonzero counts
// to the global ones (one atomic per key and workgroup instead of one per job: thousands of jobs of
// one block share a key, and same-address device atomics serialise).  nkeys <= lds capacity.
__global__ void __launch_bounds__(256) k_job_count(const Job* __restrict__ jobs, const uint32_t* __restrict__ pb, const uint32_t* __restrict__ pn,
                                                   uint32_t kb, uint32_t q, uint32_t classes, uint32_t nkeys, uint32_t* __restrict__ cnt)
{
    extern __shared__ uint32_t h[];
    const uint32_t b0 = pb ? dev_count(pb) : 0u, n = dev_count(pn);
    for (uint32_t c0 = b0 + blockIdx.x * JOB_CHUNK; c0 < n; c0 += gridDim.x * JOB_CHUNK)
    {
        for (uint32_t k = threadIdx.x; k < nkeys; k += 256)
            h[k] = 0;
        __syncthreads();
        const uint32_t c1 = min(n, c0 + JOB_CHUNK);
        for (uint32_t j = c0 + threadIdx.x; j < c1; j += 256)
            atomicAdd(&h[job_key(jobs[j], kb, q, classes)], 1u);
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nkeys; k += 256)
            if (h[k])
                atomicAdd(&cnt[k], h[k]);
        __syncthreads();
    }
}

// Scatter into key order: per chunk, local ranks from LDS atomics, one global cursor reservation per
// nonzero key and workgroup.  (Job order within a key only affects speed.)
__global__ void __launch_bounds__(256) k_job_scatter(const Job* __restrict__ in, const uint32_t* __restrict__ pb, const uint32_t* __restrict__ pn,
                                                     uint32_t kb, uint32_t q, uint32_t classes, uint32_t nkeys, uint32_t* __restrict__ cursor,
                                                     Job* __restrict__ out)
{
    extern __shared__ uint32_t h[];
    const uint32_t b0 = pb ? dev_count(pb) : 0u, n = dev_count(pn);
    constexpr int PT = JOB_CHUNK / 256;
    for (uint32_t c0 = b0 + blockIdx.x * JOB_CHUNK; c0 < n; c0 += gridDim.x * JOB_CHUNK)
    {
        for (uint32_t k = threadIdx.x; k < nkeys; k += 256)
            h[k] = 0;
        __syncthreads();
        uint32_t key[PT], rank[PT];
#pragma unroll
        for (int i = 0; i < PT; ++i)
        {
            const uint32_t j = c0 + threadIdx.x + i * 256;
            if (j < n)
            {
                key[i]  = job_key(in[j], kb, q, classes);
                rank[i] = atomicAdd(&h[key[i]], 1u);
            }
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nkeys; k += 256)
            if (h[k])
                h[k] = atomicAdd(&cursor[k], h[k]);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PT; ++i)
        {
            const uint32_t j = c0 + threadIdx.x + i * 256;
            if (j < n)
                out[h[key[i]] + rank[i]] = in[j];
        }
        __syncthreads();
    }
}

// MSD tile order.  A level's tiles (tile_bucket, in the order the scan reserved them) are listed
// XCD-major and block-major: the key of a tile is that of its block (job_key without size class).
// Workgroup w then works on XCD w % 8's part of the list, tiles of the blocks b = x (mod 8) in block
// order, so the digit gathers of the scatter hit the one or two blocks its XCD's L2 holds.
__device__ __forceinline__ uint32_t tile_key(uint32_t block, uint32_t kb, uint32_t q) { return (block & 7u) * kb + (block >> 3) / q; }

__global__ void __launch_bounds__(256) k_tile_count(const Bucket* __restrict__ buckets, const uint32_t* __restrict__ tile_bucket,
                                                    const uint32_t* __restrict__ pn, uint32_t kb, uint32_t q, uint32_t nkeys, uint32_t* __restrict__ cnt)
{
    extern __shared__ uint32_t h[];
    const uint32_t n = dev_count(pn);
    for (uint32_t c0 = blockIdx.x * JOB_CHUNK; c0 < n; c0 += gridDim.x * JOB_CHUNK)
    {
        for (uint32_t k = threadIdx.x; k < nkeys; k += 256)
            h[k] = 0;
        __syncthreads();
        const uint32_t c1 = min(n, c0 + JOB_CHUNK);
        for (uint32_t j = c0 + threadIdx.x; j < c1; j += 256)
            atomicAdd(&h[tile_key(buckets[tile_bucket[j]].block, kb, q)], 1u);
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nkeys; k += 256)
            if (h[k])
                atomicAdd(&cnt[k], h[k]);
        __syncthreads();
    }
}

// One workgroup: exclusive prefix of the key counts into cursors, per-XCD list ranges into xseg[0..8].
__global__ void __launch_bounds__(256) k_tile_prefix(const uint32_t* __restrict__ cnt, uint32_t nkeys, uint32_t kb, uint32_t* __restrict__ cursor,
                                                     uint32_t* __restrict__ xseg)
{
    __shared__ uint32_t tmp[8];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0)
        carry = 0;
    __syncthreads();
    for (uint32_t k0 = 0; k0 < nkeys; k0 += 256)
    {
        const uint32_t k = k0 + threadIdx.x;
        const uint32_t c = k < nkeys ? cnt[k] : 0u;
        uint32_t       tot;
        const uint32_t ex = block256_exclusive_sum(c, tmp, &tot) + carry;
        if (k < nkeys)
        {
            cursor[k] = ex;
            if (k % kb == 0)
                xseg[k / kb] = ex;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0)
        xseg[8] = carry;
}

// One workgroup: the job lists' key counts cnt[list][class][nk] (k_job_count) -> cursors of the same
// layout and the per-XCD ranges of the job launches, seg[16 * k + x] (x = 0..8): k = 0 the wave
// jobs (list 0, one class), k = 1 + c the workgroup jobs of size class c (list 1).  The classes of
// a list are stored one after the other.
__global__ void __launch_bounds__(256) k_job_prefix(const uint32_t* __restrict__ cnt, uint32_t nk, uint32_t kb, uint32_t classes,
                                                    uint32_t* __restrict__ cursor, uint32_t* __restrict__ seg)
{
    __shared__ uint32_t tmp[8];
    __shared__ uint32_t carry;
    for (uint32_t l = 0; l < 2; ++l)
    {
        if (threadIdx.x == 0)
            carry = 0;
        __syncthreads();
        const uint32_t nc = l == 0 ? 1u : classes;
        for (uint32_t c = 0; c < nc; ++c)
        {
            uint32_t*       xs = seg + 16 * (l == 0 ? 0 : 1 + c);
            const uint32_t* hc = cnt + ((size_t) l * MJ_CLASSES + c) * nk;
            uint32_t*       hu = cursor + ((size_t) l * MJ_CLASSES + c) * nk;
            for (uint32_t k0 = 0; k0 < nk; k0 += 256)
            {
                const uint32_t k = k0 + threadIdx.x;
                const uint32_t v = k < nk ? hc[k] : 0u;
                uint32_t       tot;
                const uint32_t ex = block256_exclusive_sum(v, tmp, &tot) + carry;
                if (k < nk)
                {
                    hu[k] = ex;
                    if (k % kb == 0)
                        xs[k / kb] = ex;
                }
                __syncthreads();
                if (threadIdx.x == 0)
                    carry += tot;
                __syncthreads();
            }
            if (threadIdx.x == 0)
                xs[8] = carry;
            __syncthreads();
        }
    }
}

__global__ void __launch_bounds__(256) k_tile_scatter(const Bucket* __restrict__ buckets, const uint32_t* __restrict__ tile_bucket,
                                                      const uint32_t* __restrict__ pn, uint32_t kb, uint32_t q, uint32_t nkeys,
                                                      uint32_t* __restrict__ cursor, const PackDesc* __restrict__ pkd,
                                                      const TileDesc* __restrict__ nat, TileDesc* __restrict__ order)
{
    extern __shared__ uint32_t h[];
    const uint32_t n = dev_count(pn);
    constexpr int PT = JOB_CHUNK / 256;
    for (uint32_t c0 = blockIdx.x * JOB_CHUNK; c0 < n; c0 += gridDim.x * JOB_CHUNK)
    {
        for (uint32_t k = threadIdx.x; k < nkeys; k += 256)
            h[k] = 0;
        __syncthreads();
        uint32_t key[PT], rank[PT];
#pragma unroll
        for (int i = 0; i < PT; ++i)
        {
            const uint32_t j = c0 + threadIdx.x + i * 256;
            if (j < n)
            {
                key[i]  = tile_key(buckets[tile_bucket[j]].block, kb, q);
                rank[i] = atomicAdd(&h[key[i]], 1u);
            }
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nkeys; k += 256)
            if (h[k])
                h[k] = atomicAdd(&cursor[k], h[k]);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PT; ++i)
        {
            const uint32_t j = c0 + threadIdx.x + i * 256;
            if (j < n)
            {
                const uint32_t  bi = tile_bucket[j];
                const Bucket    B  = buckets[bi];
                const PackDesc  P  = pkd[B.block];
                const uint32_t  f  = (j - B.tile0) * TILE;
                order[h[key[i]] + rank[i]] =
                    TileDesc{j, bi, B.start + f, min((uint32_t) TILE, B.len - f), B.d, B.start, B.len, B.buf, P.poff, P.nbits, B.kd,
                             nat[j].pdig, P.b};
            }
        }
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------------------
// fallback (prefix doubling on ranks) helpers
// -------------------------------------------------------------------------------------------------
// Copy the members of fallback groups that still live in a KV buffer into fsa.
__global__ void k_group_flush(const Group* __restrict__ groups, uint32_t ng, const uint32_t* __restrict__ p32, uint32_t* __restrict__ fsa)
{
    // (the MSD scatters leave a fallback group's payload low words in p32, by slot)
    for (uint32_t gi = blockIdx.x; gi < ng; gi += gridDim.x)
    {
        const Group G = groups[gi];
        if (G.block & (1u << 30))
            continue;
        for (uint32_t i = threadIdx.x; i < G.len; i += blockDim.x)
            fsa[G.start + i] = p32[G.start + i] & 0xFFFFFFu;
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
        {
            const uint32_t f = fsa[B.off + j];
            if (BRA_DCHECK(f < B.len, "isa_init fsa %u n %u block %u j %u", f, B.len, b, j))
                isa[B.off + f] = j;
        }
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
        {
            const uint32_t f = fsa[G.start + i];
            if (BRA_DCHECK(f < BD.len && G.start >= BD.off && G.start + G.len <= BD.off + BD.len, "group_mark fsa %u n %u start %u len %u", f,
                           BD.len, G.start, G.len))
                isa[BD.off + f] = G.start - (uint32_t) BD.off;
        }
        if (threadIdx.x == 0)
            flag[b] = 1;
    }
}

// Fallback groups from the MSD levels and the jobs carry virtual-byte depths: their members share
// 8 * depth bits of the packed string, i.e. at least floor(8 * depth / b) whole characters, the depth
// unit of the prefix doubling below (a smaller depth is still a valid one, see k_rank_keys).
__global__ void k_group_depth_chars(Group* __restrict__ groups, uint32_t ng, const PackDesc* __restrict__ pkd)
{
    for (uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x; gi < ng; gi += gridDim.x * blockDim.x)
        groups[gi].depth = (uint32_t) ((8ull * groups[gi].depth) / pkd[groups[gi].block & 0x3FFFFFFFu].b);
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
            uint32_t       idx = fsa[s];
            if (!BRA_DCHECK(idx < BD.len && s >= BD.off && s < BD.off + BD.len, "rank_keys idx %u n %u slot %u", idx, BD.len, s))
                idx = 0;
            uint32_t q = idx + h;
            if (q >= BD.len)
                q -= BD.len;
            const uint32_t rk = isa[BD.off + q];
            key0[s]           = (uint64_t) rk << 32;
            const uint32_t pv = (idx == 0) ? BD.len - 1 : idx - 1;
            pay0[s]           = ((uint32_t) in[BD.off + pv] << 24) | idx;
        }
    }
}

// Groups -> RANK buckets (big; tiles reserved for the first level), one workgroup job per medium
// group, one wave job per small group.
__global__ void k_groups_to_work(const Group* __restrict__ groups, uint32_t ng, Bucket* __restrict__ big, uint32_t cap_big,
                                 uint32_t* __restrict__ tile_bucket, uint32_t cap_tiles, Job* __restrict__ jobs, uint32_t cap_jobs,
                                 Job* __restrict__ mjobs, uint32_t cap_mjobs, uint32_t mjob_max, Counters* __restrict__ ctr,
                                 Counters* __restrict__ lout)
{
    for (uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x; gi < ng; gi += gridDim.x * blockDim.x)
    {
        const Group    G = groups[gi];
        const uint32_t b = G.block & 0x3FFFFFFFu;
        if (G.len > mjob_max)
        {
            const uint32_t ntl = div_up(G.len, TILE);
            const unsigned long long old =
                atomicAdd(reinterpret_cast<unsigned long long*>(&lout->n_big), ((unsigned long long) ntl << 32) | 1ull);
            const uint32_t s = (uint32_t) old, t0 = (uint32_t) (old >> 32);
            if (s < cap_big && t0 + ntl <= cap_tiles)
            {
                big[s] = Bucket{G.start, G.len, 0, 0, b, 0, G.depth, t0};
                for (uint32_t t = 0; t < ntl; ++t)
                    tile_bucket[t0 + t] = s;
            }
            else
                atomicExch(&ctr->overflow, 1u);
        }
        else if (G.len > JOB_MAX)
        {
            const uint32_t s = atomicAdd(&ctr->n_mjobs, 1u);
            if (s < cap_mjobs)
                mjobs[s] = Job{G.start, G.len, 0, 0, b, G.depth, 0};
            else
                atomicExch(&ctr->overflow, 1u);
        }
        else
        {
            const uint32_t s = atomicAdd(&ctr->n_jobs, 1u);
            if (s < cap_jobs)
                jobs[s] = Job{G.start, G.len, 0, 0, b, G.depth, 0};
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
// The job launches of a STRING encode (kept for the job-phase re-runs of bra_gpu_debug_rerun_jobs).
struct JobPhase
{
    JobArgs  ja, jm;
    uint32_t nblocks;
};

struct BwtWorkspace
{
    uint64_t  cap_n          = 0;
    uint32_t  cap_blocks     = 0;
    uint64_t* key[2]         = {nullptr, nullptr};
    uint32_t* p32            = nullptr;  // STRING: payload low words of the elements that leave the levels for jobs / fallback groups
    uint32_t* pay[2]         = {nullptr, nullptr};
    uint32_t* fsa            = nullptr;
    uint32_t* isa            = nullptr;
    uint32_t* tile_hist      = nullptr;
    uint32_t* tile_off       = nullptr;
    uint32_t* tile_bucket[2] = {nullptr, nullptr};
    uint8_t*  nomove         = nullptr;
    uint8_t*  flag           = nullptr;
    Bucket*   big[2]         = {nullptr, nullptr};
    Bucket*   l0b            = nullptr;  // level-0 buckets (one per block), kept for the cached geometry
    Job*      jobs           = nullptr;
    Job*      mjobs          = nullptr;
    Job*      jobs_sorted    = nullptr;  // block-major, XCD-major copies (order_jobs)
    Job*      mjobs_sorted   = nullptr;
    uint32_t* job_cnt        = nullptr;  // 2 lists x MJ_CLASSES size classes x 8 * ceil(blocks / 8) keys, then the cursors
    uint32_t* jseg           = nullptr;  // per-XCD ranges of the job launches (k_job_prefix), (1 + MJ_CLASSES) x 16 dwords
    uint32_t* tile_cnt       = nullptr;  // MSD tile order: key counts, cursors, xseg[9]
    TileDesc* tile_order     = nullptr;
    TileDesc* tdesc[2]       = {nullptr, nullptr};  // STRING: tile-order descriptors written by the scan (per level, ping-pong)
    uint8_t*  dig[2]         = {nullptr, nullptr};  // STRING: digit of the current level beside each payload of key[b]
    Group*    groups[2]      = {nullptr, nullptr};
    Counters* ctr            = nullptr;  // MAX_LEVELS slots: [0] call-wide lists, [k] level k's buckets
    Counters* h_ctr          = nullptr;  // pinned copy (byte accounting when profiling)
    Mail*     h_mail         = nullptr;  // pinned, device-written mailbox records (one per level slot)
    uint32_t  mail_seq       = 0;
    uint32_t  jobs_seq       = 0;        // the mailbox record posted right after an encode's jobs (bwt_encode_finish waits for it)
    L0Tile*   l0tiles        = nullptr;
    uint8_t*  packed         = nullptr;  // packed key strings (PackDesc.poff), N + PACK_PAD per block
    PackDesc* pkd            = nullptr;  // per block
    uint32_t* amask          = nullptr;  // per block: 256-bit presence mask of the byte values
    uint32_t* tmask          = nullptr;  // per level-0 tile: the same mask
    uint32_t* l0tot          = nullptr;  // per block: level-0 digit totals (k_l0_colscan)
    uint32_t* l0base         = nullptr;  // per block: level-0 sub-bucket starts (k_scan)
    std::vector<BlockDesc> geo;          // block geometry the level-0 tiles / buckets on the device were built for
    uint32_t  nt0 = 0;
    uint32_t  cap_tiles = 0, cap_big = 0, cap_jobs = 0, cap_mjobs = 0, cap_groups = 0, cap_l0 = 0;
    int       grid       = 16384;     // workgroups of the MSD / level-0 tile kernels (2048: 11.9, 8192: 12.3, 16384: 12.5 GB/s)
    uint32_t  scan_grid  = 4096;      // workgroups of a level's scan (4 buckets each per pass)
    uint32_t  lookahead  = 2;         // MSD levels enqueued before the host has seen the bucket count they consume
    int       mj_waves   = MJ_WAVES_DEF;  // waves of the largest workgroup job (0: no workgroup jobs)
    uint32_t  jobs_grid  = 2048;      // workgroups of the wave-job launch: about the resident capacity (with the
                                      // dynamic job queues extra groups only cost launch overhead: 8192: 2.94 ms, 2048: 2.67)
    uint32_t* jobq       = nullptr;   // per-XCD claim counters of the job launches ((1 + MJ_CLASSES) x 8 x 32 dwords)
    uint32_t  jobq_chunk = JQ_CHUNK;  // wave jobs claimed at once
    uint32_t  nblocks    = 0;         // blocks of the current call
    uint32_t  levels     = 0;         // MSD levels enqueued by the last STRING level loop
    JobPhase  last_ph{};                // job launches and batch size of the last STRING encode (diagnostics)
    uint64_t  last_n     = 0;         // 0: no job phase to re-run (none yet, a fallback rewrote the lists, or another call ran since)
    uint32_t* audit_cnt  = nullptr;   // slot-cover counts of the job audit (allocated on first use)
    uint64_t  audit_cap  = 0;
    uint32_t  mj_classes() const { return mj_waves >= 4 ? 2u : 1u; }
    uint32_t  mjob_max() const { return mj_waves ? 256u * (uint32_t) mj_waves : JOB_MAX; }
};

// ---- host mailbox ----
// k_publish writes the call counters and one level slot into a pinned record; the host spins on the
// record's sequence number.  Nothing is copied and the stream is not synchronised, so the device
// keeps running the levels enqueued ahead while the host reads.
static uint32_t post(BwtWorkspace& w, uint32_t slot, hipStream_t s)
{
    if (++w.mail_seq == 0)
        w.mail_seq = 1;
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, w.ctr, slot ? w.ctr + slot : nullptr, w.h_mail + slot, w.mail_seq);
    return w.mail_seq;
}

static bool wait_mail(BwtWorkspace& w, uint32_t slot, uint32_t seq, hipStream_t s, Mail& out)
{
    Mail* m = w.h_mail + slot;
    for (uint32_t i = 1;; ++i)
    {
        if (__atomic_load_n(&m->seq, __ATOMIC_ACQUIRE) == seq)
        {
            out.n_big    = __atomic_load_n(&m->n_big, __ATOMIC_RELAXED);
            out.n_tiles  = __atomic_load_n(&m->n_tiles, __ATOMIC_RELAXED);
            out.overflow = __atomic_load_n(&m->overflow, __ATOMIC_RELAXED);
            out.n_groups = __atomic_load_n(&m->n_groups, __ATOMIC_RELAXED);
            out.hmin     = __atomic_load_n(&m->hmin, __ATOMIC_RELAXED);
            out.n_jobs   = __atomic_load_n(&m->n_jobs, __ATOMIC_RELAXED);
            out.n_mjobs  = __atomic_load_n(&m->n_mjobs, __ATOMIC_RELAXED);
            out.n_melems = __atomic_load_n(&m->n_melems, __ATOMIC_RELAXED);
            out.seq      = seq;
            if (out.overflow)
            {
                bra_hip_report("bwt: work list overflow");
                return false;
            }
            return true;
        }
        if ((i & 255) == 0)
        {
            // a launch failed or the stream drained without the record: report instead of spinning forever
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess && __atomic_load_n(&m->seq, __ATOMIC_ACQUIRE) != seq)
            {
                bra_hip_report("bwt: mailbox record %u never arrived", slot);
                return false;
            }
            if (q != hipSuccess && q != hipErrorNotReady)
            {
                bra_hip_report("bwt: stream error while waiting for level counts: %s", hipGetErrorString(q));
                return false;
            }
        }
        __builtin_ia32_pause();
    }
}

static bool post_wait(BwtWorkspace& w, uint32_t slot, hipStream_t s, Mail& out)
{
    const uint32_t seq = post(w, slot, s);
    return wait_mail(w, slot, seq, s, out);
}

// Reorder the wave-job and workgroup-job lists block-major per XCD (see job_range), all on the
// device: count jobs per key, k_job_prefix (cursors + the launches' per-XCD ranges), scatter.  The
// workgroup jobs are also split into size classes (mjob_class): out[0] wave jobs, out[1 + c] the
// workgroup jobs of class c.  The job counts are read on the device (counters slot 0), so the host
// never waits for them.
static bool order_jobs(BwtWorkspace& w, uint32_t nblocks, const JobArgs& ja, const JobArgs& jm, JobArgs (&out)[1 + MJ_CLASSES], hipStream_t s)
{
    const uint32_t  kb0 = div_up(nblocks, 8), q = div_up(kb0, 512u);
    const uint32_t  kb = div_up(kb0, q), nk = 8 * kb;  // keys per size class (<= 4096)
    const uint32_t  classes[2] = {1, w.mj_classes()};
    const Job*      src[2]     = {w.jobs, w.mjobs};
    Job*            dst[2]     = {w.jobs_sorted, w.mjobs_sorted};
    const uint32_t* pn[2]      = {&w.ctr[0].n_jobs, &w.ctr[0].n_mjobs};
    uint32_t*       dcnt       = w.job_cnt;                                // [list][class][nk] counts
    uint32_t*       dcur       = w.job_cnt + 2 * MJ_CLASSES * (size_t) nk;  // cursors, same layout
    const dim3      g(1024);
    BRA_HIP_CHECK(hipMemsetAsync(dcnt, 0, 2 * MJ_CLASSES * (size_t) nk * 4, s));
    for (int l = 0; l < 2; ++l)
    {
        hipLaunchKernelGGL(k_job_count, g, dim3(256), classes[l] * nk * 4, s, src[l], nullptr, pn[l], kb, q, classes[l], classes[l] * nk,
                           dcnt + (size_t) l * MJ_CLASSES * nk);
        BRA_DSYNC(s);
    }
    hipLaunchKernelGGL(k_job_prefix, dim3(1), dim3(256), 0, s, dcnt, nk, kb, classes[1], dcur, w.jseg); BRA_DSYNC(s);
    for (int l = 0; l < 2; ++l)
    {
        hipLaunchKernelGGL(k_job_scatter, g, dim3(256), classes[l] * nk * 4, s, src[l], nullptr, pn[l], kb, q, classes[l], classes[l] * nk,
                           dcur + (size_t) l * MJ_CLASSES * nk, dst[l]);
        BRA_DSYNC(s);
    }
    for (uint32_t k = 0; k < 1 + MJ_CLASSES; ++k)
    {
        out[k]           = k == 0 ? ja : jm;
        out[k].jobs      = k == 0 ? dst[0] : dst[1];
        out[k].xcd_major = 1;
        out[k].dxseg     = w.jseg + 16 * k;
        out[k].njobs     = 0;  // unknown on the host; the launches read the ranges from dxseg
    }
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

static uint32_t round8(uint32_t g) { return (g + 7u) & ~7u; }

template <uint32_t MODE>
static void launch_mjobs(int waves, uint32_t n, const JobArgs& a, hipStream_t s)
{
    // about the resident capacity: 6144 waves (24 per CU)
    const uint32_t cap = 6144u / (uint32_t) waves;
    const dim3     g(round8(std::min<uint32_t>(n, cap)));
    if (waves == 4)
        hipLaunchKernelGGL((k_mjobs<MODE, 4>), g, dim3(64 * 4), sizeof(JobLds<4>) + 16, s, a);
    else
        hipLaunchKernelGGL((k_mjobs<MODE, 2>), g, dim3(64 * 2), sizeof(JobLds<2>) + 16, s, a);
#ifdef BRA_DEBUG
    if (hipStreamSynchronize(s) != hipSuccess)
        fprintf(stderr, "[bra dsync] k_mjobs mode %u waves %d n %u xcd_major %u failed\n", MODE, waves, n, a.xcd_major);
#endif
}

static void ws_free(BwtWorkspace& w)
{
    for (int i = 0; i < 2; ++i)
    {
        (void) hipFree(w.key[i]);
        (void) hipFree(w.pay[i]);
        (void) hipFree(w.big[i]);
        (void) hipFree(w.groups[i]);
        (void) hipFree(w.tile_bucket[i]);
        (void) hipFree(w.tdesc[i]);
        (void) hipFree(w.dig[i]);
    }
    void* dev[] = {w.fsa,      w.isa,   w.p32,   w.tile_hist, w.tile_off, w.nomove, w.flag, w.jobs, w.mjobs, w.jobs_sorted, w.mjobs_sorted,
                   w.job_cnt,  w.jseg,  w.tile_cnt,  w.tile_order, w.ctr,  w.jobq,  w.l0tiles, w.l0b, w.packed, w.pkd, w.amask, w.tmask, w.l0tot, w.l0base,
                   w.audit_cnt};
    for (void* p : dev)
        (void) hipFree(p);
    if (w.h_ctr)
        (void) hipHostFree(w.h_ctr);
    if (w.h_mail)
        (void) hipHostFree(w.h_mail);
    // The mailbox sequence survives a reallocation: a new pinned record block can be the memory of
    // the old one (the host allocator reuses it) with the old records still in it, and a counter that
    // restarted at 1 would meet their sequence numbers again -- wait_mail then took a stale record
    // for the device's answer (order- and timing-dependent wrong level counts / fallback groups).
    const uint32_t seq = w.mail_seq;
    w                  = BwtWorkspace{};
    w.mail_seq         = seq;
}

BwtWorkspace* bwt_workspace_create() { return new BwtWorkspace(); }
const uint32_t* bwt_alpha_masks(const BwtWorkspace* w) { return w ? w->amask : nullptr; }
const uint32_t* bwt_sa(const BwtWorkspace* w) { return w ? w->fsa : nullptr; }
void            bwt_forget_jobs(BwtWorkspace* w)
{
    if (w)
        w->last_n = 0;
}
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
    w.cap_l0     = (uint32_t) (N / TILE + B + 1);
    w.cap_big    = (uint32_t) (N / JOB_MAX + B + 16);
    w.cap_tiles  = (uint32_t) (N / TILE + w.cap_big + 16);
    // Worst cases: every fallback group has >= 2 members and the groups of one list are disjoint, so
    // a list holds <= N/2 of them (a duplicated region longer than the refinement cap emits about one
    // 2-member group per byte); the fallback turns every group of <= JOB_MAX members into one wave
    // job, so the unsorted wave-job list needs N/2 entries too.  The main path's wave jobs pack
    // runs of small sub-buckets (<= N/128 + N/129 jobs), so the XCD-sorted copy stays at N/8.
    w.cap_jobs   = (uint32_t) (N / 2 + B + 1024);
    w.cap_groups = (uint32_t) (N / 2 + B + 64);
    w.cap_mjobs  = (uint32_t) (N / JOB_MAX + B + 64);
    const uint32_t cap_sorted = (uint32_t) (N / 8 + B + 1024);
    bool ok = true;
    for (int i = 0; i < 2 && ok; ++i)
        ok = dev_alloc(w.key[i], N) && dev_alloc(w.pay[i], N) && dev_alloc(w.big[i], w.cap_big) && dev_alloc(w.groups[i], w.cap_groups) &&
             dev_alloc(w.tile_bucket[i], w.cap_tiles) && dev_alloc(w.tdesc[i], w.cap_tiles) && dev_alloc(w.dig[i], N + 16);
    const uint32_t tmax  = std::max(w.cap_tiles, w.cap_l0);
    const size_t   nkeys = 8 * (size_t) div_up(B, 8);
    ok = ok && dev_alloc(w.fsa, N) && dev_alloc(w.isa, N) && dev_alloc(w.p32, N) && dev_alloc(w.tile_hist, (uint64_t) tmax * 256) &&
         dev_alloc(w.tile_off, (uint64_t) tmax * 256) && dev_alloc(w.nomove, std::max<uint32_t>(w.cap_big, B)) && dev_alloc(w.flag, B) &&
         dev_alloc(w.jobs, w.cap_jobs) && dev_alloc(w.mjobs, w.cap_mjobs) && dev_alloc(w.jobs_sorted, cap_sorted) &&
         dev_alloc(w.mjobs_sorted, w.cap_mjobs) && dev_alloc(w.job_cnt, 4 * MJ_CLASSES * nkeys) && dev_alloc(w.jseg, (1 + MJ_CLASSES) * 16) &&
         dev_alloc(w.tile_cnt, 2 * nkeys + 16) && dev_alloc(w.tile_order, w.cap_tiles) && dev_alloc(w.ctr, MAX_LEVELS) &&
         dev_alloc(w.jobq, (1 + MJ_CLASSES) * 8 * 32) && dev_alloc(w.l0tiles, w.cap_l0) && dev_alloc(w.l0b, B) &&
         dev_alloc(w.packed, N + (uint64_t) PACK_PAD * B + 128) && dev_alloc(w.pkd, B) && dev_alloc(w.amask, 8ull * B) &&
         dev_alloc(w.tmask, 8ull * w.cap_l0) && dev_alloc(w.l0tot, 256ull * B) && dev_alloc(w.l0base, 256ull * B);
    if (ok && hipHostMalloc(&w.h_ctr, MAX_LEVELS * sizeof(Counters), hipHostMallocDefault) != hipSuccess)
        w.h_ctr = nullptr, ok = false;
    if (ok && hipHostMalloc(&w.h_mail, MAX_LEVELS * sizeof(Mail), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
        w.h_mail = nullptr, ok = false;
    if (ok)
        std::memset(w.h_mail, 0, MAX_LEVELS * sizeof(Mail));  // no record left from an earlier owner of the memory (seq 0 is never posted)
    if (!ok)
    {
        (void) hipGetLastError();
        bra_hip_report("bwt: workspace allocation for %llu elements failed", (unsigned long long) N);
        ws_free(w);  // capacities back to zero: the next call retries the allocation
            return false;
    }
    std::memset(w.h_mail, 0, MAX_LEVELS * sizeof(Mail));
    w.cap_n      = N;
    w.cap_blocks = B;
    return true;
}

static size_t tile_stage_bytes() { return sizeof(TileStage); }

// The STRING jobs of a call, after the last MSD level: order the jobs block-major per XCD, then
// the wave-job launch and one workgroup-job launch per size class.  Jobs are final when emitted:
// no later level touches their slots.

static bool run_jobs(BwtWorkspace& w, const JobPhase& ph, hipStream_t s)
{
    JobArgs ord[1 + MJ_CLASSES];
    if (!order_jobs(w, ph.nblocks, ph.ja, ph.jm, ord, s))
        return false;
    BRA_HIP_CHECK(hipMemsetAsync(w.jobq, 0, (1 + MJ_CLASSES) * 8 * 32 * 4, s));
    for (uint32_t k = 0; k < 1 + MJ_CLASSES; ++k)
    {
        ord[k].jq       = w.jobq + k * 8 * 32;
        ord[k].jq_chunk = w.jobq_chunk;
    }
    {
        BRA_PROF(P_BWT_JOBS, s);
        hipLaunchKernelGGL(k_jobs<MODE_STRING>, dim3(round8(w.jobs_grid)), dim3(256), 0, s, ord[0]);
        BRA_DSYNC(s);
    }
    {
        BRA_PROF(P_BWT_MJOBS, s);
        for (uint32_t c = 0; c < w.mj_classes(); ++c)
        {
            launch_mjobs<MODE_STRING>(2 << c, ~0u, ord[1 + c], s);
            BRA_DSYNC(s);
        }
    }
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

// MSD levels for the buckets listed in counters slot 1 (w.big[cur], tiles in w.tile_bucket[cur]);
// the caller has posted slot 1's mailbox record.  Level k (k >= 1) consumes slot k and fills slot
// k + 1.  Every level's kernels read their counts on the device, so the host only decides when to
// stop: it enqueues up to `lookahead` levels beyond the last slot it has read; once a read slot is
// empty, the levels already enqueued after it find nothing to do and return at once.
// Sub-buckets become jobs / fallback groups (appended to the call-wide lists, slot 0).
// Workgroups of a level's scan; BRA_SCAN_GRID overrides (measurement).
static uint32_t scan_grid_setting(uint32_t dflt)
{
    static const uint32_t v = [dflt] {
        const char* e = getenv("BRA_SCAN_GRID");
        return e ? std::max<uint32_t>(64u, (uint32_t) atoi(e)) : dflt;
    }();
    return v;
}

// Workgroups of the level kernels (histogram, scatter); BRA_LEVEL_GRID overrides (measurement).
static int level_grid(int dflt)
{
    static const int v = [dflt] {
        const char* e = getenv("BRA_LEVEL_GRID");
        return e ? std::max(64, atoi(e)) : dflt;
    }();
    return v;
}

template <uint32_t MODE>
static bool run_levels(BwtWorkspace& w, const uint8_t* d_in, const BlockDesc* d_blocks, int cur, Group* groups_out, hipStream_t s,
                       uint32_t first_seq)
{
    const size_t   lds    = tile_stage_bytes();
    const int      grid   = level_grid(w.grid);
    const uint32_t max_lv = (MODE == MODE_STRING) ? DCAP_BIG : RANK_KEYBYTES;  // the scans emit no bucket deeper than this
    uint32_t       seqs[MAX_LEVELS + 1] = {};
    seqs[1]                             = first_seq;
    // STRING levels start at depth 1 with payloads carrying digits [1, 1 + CARRY); a level whose
    // scatter re-gathers digits (once per CARRY levels) lists its tiles XCD-major and block-major
    // (the gathers then stay in the XCD's L2); the other levels only stream payloads and take the
    // scan's tile-order descriptors as they are (no ordering kernels).
    uint32_t lvl_kd = 1;
    uint32_t k = 1, known = 0, nb_known = 1;
    while (true)
    {
        if (known > 0 && nb_known == 0)
            break;  // slot `known` is empty: level `known` and every later one have nothing to do
        if (k <= max_lv && k <= known + w.lookahead)
        {
            const uint32_t  lvl_d   = k;
            const bool      rg      = lvl_d + 1 - lvl_kd >= CARRY;
            const bool      ordered = rg;
            const Counters* lin     = w.ctr + k;
            Counters*       lout    = w.ctr + k + 1;
            TileOrder       to{nullptr, nullptr, 0};
            if (MODE == MODE_STRING && !ordered)
                to = TileOrder{w.tdesc[cur], nullptr, 1};
            else if (MODE == MODE_STRING)
            {
                // XCD-major, block-major tile list (the scatter's digit gathers stay in the XCD's L2)
                const uint32_t kb0 = div_up(w.nblocks, 8), q = div_up(kb0, 1024u), kb = div_up(kb0, q), nk = 8 * kb;
                uint32_t*      cnt = w.tile_cnt, *cur_ = w.tile_cnt + nk, *xs = w.tile_cnt + 2 * nk;
                const dim3     g(1024);
                BRA_HIP_CHECK(hipMemsetAsync(cnt, 0, nk * 4, s));
                hipLaunchKernelGGL(k_tile_count, g, dim3(256), nk * 4, s, w.big[cur], w.tile_bucket[cur], &lin->n_tiles_next, kb, q, nk, cnt);
                BRA_DSYNC(s);
                hipLaunchKernelGGL(k_tile_prefix, dim3(1), dim3(256), 0, s, cnt, nk, kb, cur_, xs); BRA_DSYNC(s);
                hipLaunchKernelGGL(k_tile_scatter, g, dim3(256), nk * 4, s, w.big[cur], w.tile_bucket[cur], &lin->n_tiles_next, kb, q, nk, cur_,
                                   w.pkd, w.tdesc[cur], w.tile_order);
                BRA_DSYNC(s);
                to = TileOrder{w.tile_order, xs, 0};
            }
            {
                BRA_PROF(P_BWT_HIST, s);
                hipLaunchKernelGGL(k_hist<MODE>, dim3(grid), dim3(TPB), 0, s, w.big[cur], w.tile_bucket[cur], w.key[0], w.key[1], w.pay[0],
                                   w.pay[1], w.tile_hist, lin, to, w.dig[0], w.dig[1]); BRA_DSYNC(s);
            }
            ScanArgs a{d_blocks, w.big[cur],  0,           w.tile_hist, w.tile_off,  w.nomove,     w.big[cur ^ 1],
                       w.cap_big,   w.tile_bucket[cur ^ 1],   w.tdesc[cur ^ 1], w.cap_tiles, w.jobs,       w.cap_jobs,
                       w.mjobs,     w.cap_mjobs, groups_out,  w.cap_groups, w.ctr, MODE == MODE_STRING ? DCAP_BIG : RANK_KEYBYTES,
                       (uint32_t) (g_prof != nullptr), w.mjob_max(), lin, lout, w.pkd, nullptr, nullptr,
};
            {
                BRA_PROF(P_BWT_SCAN, s);
                hipLaunchKernelGGL(k_scan<MODE>, dim3(scan_grid_setting(w.scan_grid)), dim3(64 * SCAN_WAVES), 0, s, a); BRA_DSYNC(s);
            }
            {
                BRA_PROF(P_BWT_SCATTER, s);
                if (MODE == MODE_STRING)
                    hipLaunchKernelGGL(k_scatter_p, dim3(grid), dim3(TPB), sizeof(TileStageS), s, w.packed, w.nomove, w.tile_off, w.key[0],
                                       w.key[1], lin, to, w.dig[0], w.dig[1], w.p32);
                else
                    hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(TPB), lds, s, w.big[cur], w.nomove, w.tile_bucket[cur], lin, w.tile_off,
                                       w.key[0], w.key[1], w.pay[0], w.pay[1], MODE);
                BRA_DSYNC(s);
            }
            BRA_HIP_CHECK(hipGetLastError());
            seqs[k + 1] = post(w, k + 1, s);
            cur ^= 1;
            if (rg)
                lvl_kd = lvl_d + 1;
            ++k;
            continue;
        }
        Mail m{};
        if (!wait_mail(w, known + 1, seqs[known + 1], s, m))
            return false;
        ++known;
        nb_known = m.n_big;
        if (known > max_lv)
            break;
    }
    w.levels = k - 1;
    return true;
}

// Algorithmic bytes of the MSD levels (profiling only: one copy of the level counters).
template <uint32_t MODE>
static bool account_levels(BwtWorkspace& w, hipStream_t s)
{
    if (!g_prof || !(g_prof->mask >> P_BWT_HIST & 1 || g_prof->mask >> P_BWT_SCAN & 1 || g_prof->mask >> P_BWT_SCATTER & 1))
        return true;
    const uint32_t ns = std::min<uint32_t>(w.levels + 2, MAX_LEVELS);
    BRA_HIP_CHECK(hipMemcpyAsync(w.h_ctr, w.ctr, ns * sizeof(Counters), hipMemcpyDeviceToHost, s));
    BRA_HIP_CHECK(hipStreamSynchronize(s));
    // STRING: 8-byte payloads moved (+ the next digit gathered for elements that stay in big buckets);
    // elements leaving for a job write a 4-byte word instead, so this is an upper estimate
    const double eb = 8.0, mb = (MODE == MODE_STRING) ? 16.0 + 8.0 / CARRY : 24.0;
    for (uint32_t k = 1; k + 1 < ns; ++k)
    {
        const Counters& c  = w.h_ctr[k];
        const double    nt = c.n_tiles_next, ne = c.n_elems_next, nm = w.h_ctr[k + 1].n_moved;
        if (c.n_big == 0)
            break;
        prof_bytes(P_BWT_HIST, eb * ne + 1024.0 * nt);
        prof_bytes(P_BWT_SCAN, 3072.0 * nt + 32.0 * c.n_big);
        prof_bytes(P_BWT_SCATTER, mb * nm + 1024.0 * nt);
    }
    return true;
}

// The job audit (k_audit_cover / k_audit_check) of the jobs in the lists; returns the number of
// failing jobs (-1 on a HIP error).
static int audit_jobs(BwtWorkspace& w, uint64_t N, const BlockDesc* d_blocks, hipStream_t s)
{
    if (N > w.audit_cap)
    {
        (void) hipFree(w.audit_cnt);
        w.audit_cnt = nullptr;
        w.audit_cap = 0;
        if (hipMalloc(&w.audit_cnt, N * 4) != hipSuccess)
            return -1;
        w.audit_cap = N;
    }
    uint32_t* const cnt = w.audit_cnt;
    static const uint32_t zero = 0;
    uint32_t              fails = 0;
    if (hipMemsetAsync(cnt, 0, N * 4, s) != hipSuccess ||
        hipMemcpyToSymbolAsync(HIP_SYMBOL(g_audit_prints), &zero, 4, 0, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyToSymbolAsync(HIP_SYMBOL(g_audit_fail), &zero, 4, 0, hipMemcpyHostToDevice, s) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_audit_cover, dim3(4096), dim3(256), 0, s, w.jobs, &w.ctr[0].n_jobs, cnt);
    hipLaunchKernelGGL(k_audit_cover, dim3(4096), dim3(256), 0, s, w.mjobs, &w.ctr[0].n_mjobs, cnt);
    hipLaunchKernelGGL(k_audit_check, dim3(4096), dim3(256), 0, s, w.jobs, &w.ctr[0].n_jobs, 0u, w.p32, w.fsa, cnt, d_blocks);
    hipLaunchKernelGGL(k_audit_check, dim3(4096), dim3(256), 0, s, w.mjobs, &w.ctr[0].n_mjobs, 1u, w.p32, w.fsa, cnt, d_blocks);
    if (hipStreamSynchronize(s) != hipSuccess || hipMemcpyFromSymbol(&fails, HIP_SYMBOL(g_audit_fail), 4) != hipSuccess)
        return -1;
#ifdef BRA_JOB_AUDIT
    uint32_t sf = 0;
    if (hipMemcpyFromSymbol(&sf, HIP_SYMBOL(g_sort_fail), 4) != hipSuccess)
        return -1;
    if (sf)
    {
        static bool dumped = false;
        fprintf(stderr, "[bwt audit] %u job sorts not ascending\n", sf);
        if (!dumped)
        {
            dumped = true;
            static uint64_t dump[2][1024];
            uint32_t        meta[4];
            if (hipMemcpyFromSymbol(dump, HIP_SYMBOL(g_sort_dump), sizeof dump) == hipSuccess &&
                hipMemcpyFromSymbol(meta, HIP_SYMBOL(g_sort_meta), sizeof meta) == hipSuccess)
            {
                const char* dir = getenv("BRA_DIAG_DIR");
                char        path[512];
                snprintf(path, sizeof path, "%s/sort_dump.bin", dir ? dir : ".");
                static uint64_t phases[10][1024];
                if (hipMemcpyFromSymbol(phases, HIP_SYMBOL(g_sort_phase), sizeof phases) != hipSuccess)
                    return -1;
                if (FILE* f = fopen(path, "wb"))
                {
                    fwrite(meta, 4, 4, f);
                    fwrite(dump, 8, 2 * 1024, f);
                    fwrite(phases, 8, 10 * 1024, f);
                    fclose(f);
                    fprintf(stderr, "[bwt audit] first failing sort (W %u, P %u, xcc %u) dumped to %s\n", meta[0], meta[1], meta[2], path);
                }
            }
        }
        const uint32_t z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sort_fail), &z, 4) != hipSuccess)
            return -1;
    }
#endif
    return (int) fails;
}

// Re-runs the job phase of the last STRING encode `reps` times on the unchanged lists and payloads
// (the jobs only read them) and audits every run; returns the failing jobs summed over the runs.
// Valid only right after a STRING encode on this workspace whose input buffer the caller still
// holds (the job launches read it); -1 when there is nothing to re-run.
int bwt_debug_rerun_jobs(BwtWorkspace* wp, int reps, hipStream_t s, uint32_t seed)
{
    if (!wp->last_n || reps < 0)
        return -1;
    int total = 0;
    for (int r = 0; r < reps; ++r)
    {
        if (seed)
        {
            hipLaunchKernelGGL(k_audit_shuffle, dim3(4096), dim3(1024), 0, s, wp->jobs, &wp->ctr[0].n_jobs, wp->p32, seed + (uint32_t) r);
            hipLaunchKernelGGL(k_audit_shuffle, dim3(4096), dim3(1024), 0, s, wp->mjobs, &wp->ctr[0].n_mjobs, wp->p32, seed + (uint32_t) r);
        }
        if (!run_jobs(*wp, wp->last_ph, s))
            return -1;
        const int f = audit_jobs(*wp, wp->last_n, wp->last_ph.ja.blocks, s);
        if (f < 0)
            return -1;
        total += f;
    }
    return total;
}

bool bwt_encode_device(BwtWorkspace* wp, const uint8_t* d_in, const BlockDesc* d_blocks, const BlockDesc* h_blocks, uint32_t nblocks,
                       uint8_t* d_L, uint32_t* d_pi, hipStream_t s)
{
    return bwt_encode_enqueue(wp, d_in, d_blocks, h_blocks, nblocks, d_L, d_pi, s) &&
           bwt_encode_finish(wp, d_in, d_blocks, h_blocks, nblocks, d_L, d_pi, s, nullptr);
}

bool bwt_encode_enqueue(BwtWorkspace* wp, const uint8_t* d_in, const BlockDesc* d_blocks, const BlockDesc* h_blocks, uint32_t nblocks,
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
    w.last_n = 0;  // the job phase of an earlier encode is no longer re-runnable
    if (!ws_reserve(w, N, nblocks))
        return false;
    w.nblocks = nblocks;
#ifdef BRA_DEBUG
    // poison every work buffer so that a read of anything this call did not write shows up
    for (int i = 0; i < 2; ++i)
    {
        BRA_HIP_CHECK(hipMemsetAsync(w.key[i], 0xA5, N * 8, s));
        BRA_HIP_CHECK(hipMemsetAsync(w.pay[i], 0xA5, N * 4, s));
        BRA_HIP_CHECK(hipMemsetAsync(w.big[i], 0xA5, (size_t) w.cap_big * sizeof(Bucket), s));
        BRA_HIP_CHECK(hipMemsetAsync(w.groups[i], 0xA5, (size_t) w.cap_groups * sizeof(Group), s));
        BRA_HIP_CHECK(hipMemsetAsync(w.tile_bucket[i], 0xA5, (size_t) w.cap_tiles * 4, s));
    }
    BRA_HIP_CHECK(hipMemsetAsync(w.fsa, 0xA5, N * 4, s));
    BRA_HIP_CHECK(hipMemsetAsync(w.isa, 0xA5, N * 4, s));
    BRA_HIP_CHECK(hipMemsetAsync(w.jobs, 0xA5, (size_t) w.cap_jobs * sizeof(Job), s));
    BRA_HIP_CHECK(hipMemsetAsync(w.mjobs, 0xA5, (size_t) w.cap_mjobs * sizeof(Job), s));
    BRA_HIP_CHECK(hipMemsetAsync(w.nomove, 0xA5, std::max<uint32_t>(w.cap_big, nblocks), s));
    BRA_HIP_CHECK(hipMemsetAsync(d_L, 0xA5, N, s));
    BRA_HIP_CHECK(hipMemsetAsync(w.tile_hist, 0xA5, (size_t) std::max(w.cap_tiles, w.cap_l0) * 256 * 4, s));
    BRA_HIP_CHECK(hipMemsetAsync(w.tile_off, 0xA5, (size_t) std::max(w.cap_tiles, w.cap_l0) * 256 * 4, s));
#endif
    // kernel attributes are per device: set them once on every device this process encodes on
    static std::atomic<uint64_t> attr_set{0};
    int dev = 0;
    BRA_HIP_CHECK(hipGetDevice(&dev));
    const uint64_t dev_bit = 1ull << (dev & 63);
    if (!(attr_set.load() & dev_bit))
    {
        const size_t lds = tile_stage_bytes();
        BRA_HIP_CHECK(hipFuncSetAttribute((const void*) k_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
        BRA_HIP_CHECK(hipFuncSetAttribute((const void*) k_l0_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int) (sizeof(TileStageL0) + TILE + 64)));
        attr_set.fetch_or(dev_bit);
    }
    const int grid = w.grid;

    // ---- level 0 (buckets = blocks, elements read straight from the input) ----
    // The tile list and the per-block buckets depend only on the geometry: uploaded once per geometry.
    if (w.geo.size() != nblocks || std::memcmp(w.geo.data(), h_blocks, nblocks * sizeof(BlockDesc)) != 0)
    {
        std::vector<L0Tile> tiles;
        std::vector<Bucket> l0b(nblocks);
        for (uint32_t b = 0; b < nblocks; ++b)
        {
            l0b[b] = Bucket{(uint32_t) h_blocks[b].off, h_blocks[b].len, 0, 0, b, 2u, 0, (uint32_t) tiles.size()};
            for (uint32_t st = 0; st < h_blocks[b].len; st += TILE)
                tiles.push_back(L0Tile{b, st});
        }
        w.geo.clear();
        w.nt0 = (uint32_t) tiles.size();
        BRA_HIP_CHECK(hipMemcpyAsync(w.l0tiles, tiles.data(), w.nt0 * sizeof(L0Tile), hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipMemcpyAsync(w.l0b, l0b.data(), nblocks * sizeof(Bucket), hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipStreamSynchronize(s));  // the host vectors are the copies' sources
        w.geo.assign(h_blocks, h_blocks + nblocks);
    }
    const uint32_t nt0 = w.nt0;
    hipLaunchKernelGGL(k_ctr_init, dim3(1), dim3(1024), 0, s, w.ctr, MAX_LEVELS);
    BRA_HIP_CHECK(hipMemsetAsync(w.flag, 0, nblocks, s));
    {
        // packed key strings: alphabet per block, bits per character, the packed cyclic strings
        BRA_PROF(P_BWT_PACK, s);
        hipLaunchKernelGGL(k_alpha, dim3(std::min<uint32_t>(nt0, grid)), dim3(TPB), 0, s, d_in, d_blocks, w.l0tiles, nt0, w.tmask); BRA_DSYNC(s);
        hipLaunchKernelGGL(k_pack_desc, dim3(std::min<uint32_t>(nblocks, 4096u)), dim3(TPB), 0, s, d_blocks, w.l0b, nblocks, w.tmask, w.amask, w.pkd);
        BRA_DSYNC(s);
        hipLaunchKernelGGL(k_pack, dim3(std::min<uint32_t>(nt0, grid)), dim3(TPB), 0, s, d_in, d_blocks, w.l0tiles, nt0, w.amask, w.pkd, w.packed);
        BRA_DSYNC(s);
    }
    {
        BRA_PROF(P_BWT_L0HIST, s);
        hipLaunchKernelGGL(k_l0_hist, dim3(std::min<uint32_t>(nt0, grid)), dim3(TPB), 0, s, w.packed, d_blocks, w.pkd, w.l0tiles, nt0, w.tile_hist);
        BRA_DSYNC(s);
    }
    ScanArgs a0{d_blocks, w.l0b,     nblocks,         w.tile_hist, w.tile_off, w.nomove,   w.big[0],    w.cap_big,
                w.tile_bucket[0], w.tdesc[0], w.cap_tiles, w.jobs,     w.cap_jobs, w.mjobs,    w.cap_mjobs, w.groups[0],
                w.cap_groups,     w.ctr,       DCAP_BIG,   (uint32_t) (g_prof != nullptr), w.mjob_max(), nullptr, w.ctr + 1, w.pkd,
                w.l0tot,          w.l0base};
    {
        BRA_PROF(P_BWT_SCAN, s);
        hipLaunchKernelGGL(k_l0_colscan, dim3(std::min<uint32_t>(nblocks, 65535u)), dim3(256 * L0CS_GROUPS), 0, s, w.l0b, nblocks, w.tile_hist,
                           w.tile_off, w.l0tot);
        BRA_DSYNC(s);
        hipLaunchKernelGGL(k_scan<MODE_STRING>, dim3(std::min<uint32_t>(div_up(nblocks, SCAN_WAVES), 65535u)), dim3(64 * SCAN_WAVES), 0, s, a0); BRA_DSYNC(s);
    }
    {
        BRA_PROF(P_BWT_L0SCATTER, s);
        hipLaunchKernelGGL(k_l0_scatter, dim3(nt0 >= 8 ? std::min<uint32_t>(nt0, grid) & ~7u : nt0), dim3(TPB), sizeof(TileStageL0) + TILE + 64, s, d_in, w.amask, w.packed, d_blocks,
                           w.pkd, w.l0tiles, nt0, w.tile_off, w.l0base, w.key[0], w.dig[0], w.p32); BRA_DSYNC(s);
    }
    BRA_HIP_CHECK(hipGetLastError());
    prof_bytes(P_BWT_PACK, 3.0 * (double) N);  // input read twice, packed string written (<= N)
    prof_bytes(P_BWT_L0HIST, (double) N + 1024.0 * nt0);
    prof_bytes(P_BWT_SCAN, 3072.0 * nt0);
    prof_bytes(P_BWT_L0SCATTER, 9.0 * N + 1024.0 * nt0);  // window in, payload out
    // level-0 sub-buckets all live in KV buffer 0, their tiles in tile_bucket[0]; the jobs run after
    // the last level
    JobPhase ph;
    ph.ja = JobArgs{w.jobs,  0,     d_in,        d_blocks, w.key[0], w.key[1], w.pay[0], w.pay[1], w.fsa, d_L, d_pi,
                    w.isa,   w.groups[0], w.cap_groups, w.ctr,  DCAP_JOB, 0, 0, {}, nullptr, nullptr, 0, w.packed, w.pkd};
    ph.ja.p32  = w.p32;
    ph.jm      = ph.ja;
    ph.jm.jobs = w.mjobs;
    ph.nblocks = nblocks;
    if (!run_levels<MODE_STRING>(w, d_in, d_blocks, 0, w.groups[0], s, post(w, 1, s)))
        return false;
    if (!run_jobs(w, ph, s))
        return false;
    // posted here, waited for in bwt_encode_finish after the caller has queued its later stages:
    // the host resumes when the jobs are done, with the rest of the step still queued ahead of the
    // device (posted at the end of the chain, the host waited for the whole step and the device
    // idled while the next one was queued)
    w.jobs_seq = post(w, 0, s);
    BRA_HIP_CHECK(hipGetLastError());
    w.last_ph = ph;
    w.last_n  = N;
#ifdef BRA_JOB_AUDIT
    if (audit_jobs(w, N, d_blocks, s) < 0)
        return false;
#endif
    if (!account_levels<MODE_STRING>(w, s))
        return false;
    static const bool level_stats = getenv("BRA_LEVEL_STATS") != nullptr;  // diagnostic: per-level counts to stderr
    if (level_stats)
    {
        const uint32_t ns = std::min<uint32_t>(w.levels + 2, MAX_LEVELS);
        BRA_HIP_CHECK(hipMemcpyAsync(w.h_ctr, w.ctr, ns * sizeof(Counters), hipMemcpyDeviceToHost, s));
        BRA_HIP_CHECK(hipStreamSynchronize(s));
        const Counters& c0 = w.h_ctr[0];
        fprintf(stderr, "[bwt levels] N %llu jobs %u mjobs %u melems %u groups %u\n", (unsigned long long) N, c0.n_jobs,
                c0.n_mjobs, c0.n_melems, c0.n_groups);
        for (uint32_t k = 1; k < ns; ++k)
            fprintf(stderr, "[bwt levels] slot %u: buckets %u tiles %u elems %u moved(into) %u\n", k, w.h_ctr[k].n_big, w.h_ctr[k].n_tiles_next,
                    w.h_ctr[k].n_elems_next, w.h_ctr[k].n_moved);
    }
    return true;
}

bool bwt_encode_finish(BwtWorkspace* wp, const uint8_t* d_in, const BlockDesc* d_blocks, const BlockDesc* h_blocks, uint32_t nblocks,
                       uint8_t* d_L, uint32_t* d_pi, hipStream_t s, bool* fallback_ran)
{
    BwtWorkspace& w = *wp;
    uint64_t      N = 0;
    for (uint32_t b = 0; b < nblocks; ++b)
        N = std::max<uint64_t>(N, h_blocks[b].off + h_blocks[b].len);
    if (fallback_ran)
        *fallback_ran = false;
    Mail mc{};
    if (!wait_mail(w, 0, w.jobs_seq, s, mc))
        return false;
#ifdef BRA_JOB_TIMING
    {
        unsigned long long jt[2][32];
        BRA_HIP_CHECK(hipMemcpyFromSymbol(jt, HIP_SYMBOL(g_jt), sizeof jt));
        for (int k = 0; k < 2; ++k)
        {
            fprintf(stderr, "[job timing %s] claim %llu gather1 %llu sort1 %llu groups+out %llu regather %llu sortN %llu | sorts %llu jobs %llu | between jobs %llu\n",
                    k ? "wg" : "wave", jt[k][0], jt[k][1], jt[k][2], jt[k][3], jt[k][4], jt[k][5], jt[k][6], jt[k][7], jt[k][8]);
            fprintf(stderr, "[job sorts %s] P:", k ? "wg" : "wave");
            for (int lg = 2; lg <= 10; ++lg)
                fprintf(stderr, " %d:%llu/%llu", 1 << lg, jt[k][10 + lg], jt[k][21 + lg]);
            fprintf(stderr, "\n");
        }
        std::memset(jt, 0, sizeof jt);
        BRA_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_jt), jt, sizeof jt));
    }
#endif
    // SURVEY 8.1(d) BWT model: 11 algorithmic bytes per element (input read, SA written and
    // re-read, L gathered and written), charged to the job kernels by the elements each kind covers
    prof_bytes(P_BWT_JOBS, 11.0 * ((double) N - (double) mc.n_melems));
    prof_bytes(P_BWT_MJOBS, 11.0 * (double) mc.n_melems);

    // ---- fallback: prefix doubling on the groups still tied ----
    uint32_t ng = mc.n_groups;
    static const bool level_stats = getenv("BRA_LEVEL_STATS") != nullptr;  // diagnostic
    if (level_stats)
        fprintf(stderr, "[bwt finish] mail seq %u groups %u jobs %u mjobs %u hmin %u\n", mc.seq, mc.n_groups, mc.n_jobs, mc.n_mjobs, mc.hmin);
    if (ng == 0)
        return true;
    if (fallback_ran)
        *fallback_ran = true;
    w.last_n = 0;  // the fallback refills the job lists and counters with RANK-mode work
    BRA_PROF(P_BWT_FALLBACK, s);
    int gcur = 0;
    hipLaunchKernelGGL(k_group_depth_chars, dim3(std::min<uint32_t>(div_up(ng, 256), 4096u)), dim3(256), 0, s, w.groups[gcur], ng, w.pkd);
    BRA_DSYNC(s);
    hipLaunchKernelGGL(k_group_flush, dim3(std::min<uint32_t>(ng, 4096u)), dim3(256), 0, s, w.groups[gcur], ng, w.p32, w.fsa); BRA_DSYNC(s);
    // mark blocks, build ranks: singletons rank = own slot, group members = group start
    hipLaunchKernelGGL(k_group_mark, dim3(std::min<uint32_t>(ng, 4096u)), dim3(256), 0, s, w.groups[gcur], ng, d_blocks, w.fsa, w.isa,
                       w.flag); BRA_DSYNC(s);  // sets the flags (its rank writes are redone below)
    hipLaunchKernelGGL(k_isa_init, dim3(64, std::min<uint32_t>(nblocks, 65535u)), dim3(256), 0, s, d_blocks, w.flag, nblocks, w.fsa, w.isa); BRA_DSYNC(s);
    hipLaunchKernelGGL(k_group_mark, dim3(std::min<uint32_t>(ng, 4096u)), dim3(256), 0, s, w.groups[gcur], ng, d_blocks, w.fsa, w.isa,
                       w.flag); BRA_DSYNC(s);
    uint32_t hmin    = mc.hmin;
    for (int round = 0; round < 64 && ng > 0; ++round)
    {
        // keys for this round (every read of isa happens here, before any rank update)
        hipLaunchKernelGGL(k_rank_keys, dim3(std::min<uint32_t>(ng, 8192u)), dim3(256), 0, s, w.groups[gcur], ng, d_blocks, d_in, w.fsa,
                           w.isa, w.key[0], w.pay[0]); BRA_DSYNC(s);
        hipLaunchKernelGGL(k_ctr_init, dim3(1), dim3(1024), 0, s, w.ctr, MAX_LEVELS);
        hipLaunchKernelGGL(k_groups_to_work, dim3(std::min<uint32_t>(div_up(ng, 256), 4096u)), dim3(256), 0, s, w.groups[gcur], ng,
                           w.big[0], w.cap_big, w.tile_bucket[0], w.cap_tiles, w.jobs, w.cap_jobs, w.mjobs, w.cap_mjobs, w.mjob_max(), w.ctr,
                           w.ctr + 1); BRA_DSYNC(s);
        Group* gnext = w.groups[gcur ^ 1];
        // sort the groups by rank key: MSD levels over the 4 key bytes; equal-key sub-buckets larger
        // than a job become next-round groups directly (emitted with the parent's depth)
        if (!run_levels<MODE_RANK>(w, d_in, d_blocks, 0, gnext, s, post(w, 1, s)))
            return false;
        Mail mr{};
        if (!post_wait(w, 0, s, mr))
            return false;
        const uint32_t ng_big = mr.n_groups;
        const uint32_t nj     = mr.n_jobs;
        JobArgs jr{w.jobs, nj, d_in, d_blocks, w.key[0], w.key[1], w.pay[0], w.pay[1], w.fsa, d_L, d_pi, w.isa, gnext, w.cap_groups,
                   w.ctr,  0,  hmin, 0, {}, nullptr, nullptr, 0, w.packed, w.pkd};
        if (ng_big)
            hipLaunchKernelGGL(k_rank_flush, dim3(std::min<uint32_t>(ng_big, 4096u)), dim3(256), 0, s, gnext, ng_big, d_blocks, w.pay[0],
                               w.pay[1], w.fsa, d_L, w.isa, d_pi); BRA_DSYNC(s);
        if (nj)
            hipLaunchKernelGGL(k_jobs<MODE_RANK>, dim3(std::min<uint32_t>(div_up(nj, 4), 8192u)), dim3(256), 0, s, jr); BRA_DSYNC(s);
        const uint32_t nmj = mr.n_mjobs;
        if (nmj)
        {
            JobArgs jm2 = jr;
            jm2.jobs    = w.mjobs;
            jm2.njobs   = nmj;
            launch_mjobs<MODE_RANK>(w.mj_waves, nmj, jm2, s);
        }
        BRA_HIP_CHECK(hipGetLastError());
        Mail me{};
        if (!post_wait(w, 0, s, me))
            return false;
        uint32_t ng_new = me.n_groups;
        // the big equal-key subgroups were emitted with the parent's depth: add the round's step,
        // mark them flushed, drop groups of identical rotations (depth >= n) and find the new step
        std::vector<Group> all(ng_new);
        if (ng_new)
        {
            BRA_HIP_CHECK(hipMemcpyAsync(all.data(), gnext, ng_new * sizeof(Group), hipMemcpyDeviceToHost, s));
            BRA_HIP_CHECK(hipStreamSynchronize(s));
        }
        for (uint32_t i = 0; i < ng_big; ++i)
        {
            all[i].depth += hmin;
            all[i].block = (all[i].block & 0x3FFFFFFFu) | (1u << 30);
        }
        std::vector<Group> keep;
        keep.reserve(ng_new);
        uint32_t m = 0xFFFFFFFFu;
        for (auto& g : all)
        {
            if (g.depth >= h_blocks[g.block & 0x3FFFFFFFu].len)
                continue;  // identical rotations: final
            m = std::min(m, g.depth);
            keep.push_back(g);
        }
        ng = (uint32_t) keep.size();
        if (level_stats)
            fprintf(stderr, "[bwt fallback] round %d: big groups %u jobs %u mjobs %u -> groups %u kept %u hmin %u\n", round, ng_big, nj, nmj, ng_new, ng, m);
        if (ng)
            BRA_HIP_CHECK(hipMemcpyAsync(gnext, keep.data(), ng * sizeof(Group), hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipStreamSynchronize(s));
        hmin = m;
        gcur ^= 1;
    }
    // every group's depth grows by the round's minimum depth, so the minimum at least doubles per
    // round: 64 rounds cover any block
    if (ng > 0)
    {
        bra_hip_report("bwt: prefix doubling did not converge (%u groups left)", ng);
        return false;
    }
    hipLaunchKernelGGL(k_pi_from_isa, dim3(std::min<uint32_t>(div_up(nblocks, 256), 1024u)), dim3(256), 0, s, d_blocks, w.flag, nblocks,
                       w.isa, d_pi); BRA_DSYNC(s);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace bra

// Diagnostics: run the job sort of W waves (1, 2 or 4) on `groups` workgroups x `iters` random key
// sets (k_sortnet_test); returns the number of failing sorts, or -1 on a launch error.
// With keys (host array of 256 * waves keys in slot order, padding = all ones), every sort uses them.
extern "C" int bra_gpu_sortnet_selftest(int waves, unsigned groups, unsigned iters, unsigned seed, const unsigned long long* keys)
{
    using namespace bra;
    if ((waves != 1 && waves != 2 && waves != 4) || groups == 0)
        return -1;
    uint32_t* d = nullptr;
    uint64_t* dk = nullptr;
    uint32_t  h = 0, tfix = 0;
    int       rc = -1;
    if (hipMalloc(&d, 4) != hipSuccess)
        return -1;
    if (keys)
    {
        const size_t nk = 256u * (unsigned) waves;
        for (size_t c = 0; c < nk; ++c)
            tfix += keys[c] != ~0ull;
        if (hipMalloc(&dk, nk * 8) != hipSuccess || hipMemcpy(dk, keys, nk * 8, hipMemcpyHostToDevice) != hipSuccess)
            goto done;
    }
    if (hipMemset(d, 0, 4) == hipSuccess)
    {
        if (waves == 1)
            hipLaunchKernelGGL(k_sortnet_test<1>, dim3(groups), dim3(64), sizeof(JobLds<1>), 0, seed, iters, d, dk, tfix);
        else if (waves == 2)
            hipLaunchKernelGGL(k_sortnet_test<2>, dim3(groups), dim3(128), sizeof(JobLds<2>), 0, seed, iters, d, dk, tfix);
        else
            hipLaunchKernelGGL(k_sortnet_test<4>, dim3(groups), dim3(256), sizeof(JobLds<4>), 0, seed, iters, d, dk, tfix);
        if (hipGetLastError() == hipSuccess && hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost) == hipSuccess)
            rc = (int) std::min<uint32_t>(h, 0x7FFFFFFF);
    }
done:
    (void) hipGetLastError();
    (void) hipFree(d);
    (void) hipFree(dk);
    return rc;
}
