// rle_decode.hip -- PackBits decoding for a batch of independent blocks.
//
// Replaces bra_rle_decode / bra_rle_decode_compute_size (reference src/encoders/bra_rle.c:122-160,
// :162-224): control c >= 0 -> c+1 literal bytes follow; -127 <= c <= -1 -> the next byte repeated
// 1-c times; c == -128 -> no-op; a block truncated by the end of the stream makes the decoded size
// 0 (error).
//
// The position of each control byte depends on every earlier one: the controls form a chain
// p -> nxt(p) = p + (c+2 | 2 | 1) through the stream.  One 1024-thread workgroup decodes one block,
// a 16 KiB window of the stream at a time, one wave per 1 KiB sub-window:
//   1. every wave computes, for every position p of its sub-window, where the chain from p leaves
//      the sub-window and how many output bytes it produces on the way (pointer jumping in LDS:
//      log2 of the chain length rounds, usually 3..8);
//   2. one lane chains the 16 sub-windows from the window's entry control (16 LDS lookups);
//   3. every wave walks the chain through its sub-window from its entry (lane-exchange steps on
//      the original successors, 64 positions per register), compacts the controls on the chain
//      with their output offsets, and writes its output range: each lane finds the control of its
//      16 output bytes (binary search + forward steps) and takes them from the staged window.
// Everything stays in LDS; the next window's bytes are loaded while the current one is decoded.
//
// Few long streams (e.g. 32 blocks of 8 MiB) would leave most CUs idle, so such batches split every
// stream into segments of whole windows, one workgroup each, in three launches:
//   a. k_rled<MAP>: for each of the RD_NENT entry offsets a chain can have into the segment (the
//      last control before it steps at most 129 bytes), its exit into the next segment and its
//      output bytes -- phase 1 as above plus phase 2 run by one lane per entry;
//   b. k_rled_link: one lane per block chains its segments through the maps: every segment's
//      entry and output offset, and the decoded size / error check;
//   c. k_rled<DEC>: the decode above, each segment from its entry.
#include "prof.h"
#include "rle.h"

namespace bra {

namespace {

constexpr uint32_t RD_WAVES = 16;                   // waves per workgroup = sub-windows per window
constexpr uint32_t RD_TPB   = RD_WAVES * 64;
constexpr uint32_t RD_SUB   = 1024;                 // stream bytes per sub-window (16 per lane)
constexpr uint32_t RD_PER   = RD_SUB / 64;          // positions per lane
constexpr uint32_t RD_WIN   = RD_WAVES * RD_SUB;    // 16 KiB window
constexpr uint32_t RD_HALO  = 256;                  // a literal's payload runs up to 128 bytes past its window
constexpr uint32_t RD_LOAD  = (RD_WIN + RD_HALO) / 16;  // 16-byte loads per window (<= 2 per thread)
constexpr uint32_t RD_NENT  = 129;                  // entry offsets into a segment: [0, 128]
constexpr uint32_t PK_SH    = 11;                   // PK word: position (< RD_SUB + 129 < 2^11) | output bytes << 11
constexpr uint32_t PK_POS   = (1u << PK_SH) - 1u;
static_assert(RD_SUB + 129 <= PK_POS + 1 && (RD_SUB / 2 * 128 + 129) < (1u << (32 - PK_SH)), "PK fields");
typedef uint4 __attribute__((aligned(1))) u128_u;

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// control byte -> (stream step, output bytes)
__device__ __forceinline__ uint32_t ctl_step(uint32_t c) { return c < 128u ? c + 2u : (c > 128u ? 2u : 1u); }
__device__ __forceinline__ uint32_t ctl_prod(uint32_t c) { return c < 128u ? c + 1u : (c > 128u ? 257u - c : 0u); }

// 16 bytes of the stream at window offset q (global), zero past the end
__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ src, uint32_t size, uint32_t at)
{
    if (at + 16u <= size && (((uintptr_t) (src + at)) & 15) == 0)
        return *reinterpret_cast<const uint4*>(src + at);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < 16; ++k)
        if (at + k < size)
            w[k >> 2] |= (uint32_t) src[at + k] << (8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Segments of a batch: block b's segment j (j < nseg) starts at stream offset j * seg_bytes (a
// multiple of RD_WIN); nseg == 1: whole blocks, entry 0, the decoded size written here.
struct RledSeg
{
    uint32_t nseg, seg_bytes;
    uint2*   map;    // MAP: [(b * nseg + j) * RD_NENT + entry] = (exit offset past the segment's last window, output bytes)
    uint2*   state;  // [b * nseg + j] = (entry offset, block output offset) (k_rled_link)
};

#ifdef BRA_RLED_TIMING
// measurement build only: shader clocks of wave 0 per phase, summed over the windows (load + 1, 2, 3)
__device__ unsigned long long g_rled_t[4];
#define RT_NOW() (threadIdx.x == 0 ? (unsigned long long) clock64() : 0ull)
#else
#define RT_NOW() 0ull
#endif

template <bool MAP>
__global__ void __launch_bounds__(RD_TPB) k_rled(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_base,
                                                 const uint32_t* __restrict__ in_size, uint32_t nblocks, uint8_t* __restrict__ out,
                                                 const uint64_t* __restrict__ out_base, const uint64_t* __restrict__ out_cap,
                                                 uint32_t* __restrict__ out_size, RledSeg sg)
{
    __shared__ uint4    win4[1 + (RD_WIN + RD_HALO) / 16];  // one 16-byte pad in front: unaligned output reads start up to 15 bytes early
    // Per sub-window position: successor (sub-window position, >= len: the exit; < 2^11) | output
    // bytes to the exit << 11 (< 2^17: at most 128 per two stream bytes); later the chain's controls:
    // position | output offset << 11.  One word per position: a pointer-jumping round is one LDS read
    // and one write per position (two of each with separate successor / count arrays).
    __shared__ uint32_t PK[RD_WAVES][RD_SUB];
    __shared__ uint32_t sub_entry[RD_WAVES], sub_out[RD_WAVES], sub_tot[RD_WAVES], sub_ncon[RD_WAVES];
    __shared__ uint32_t sh_E, sh_O;
    const uint8_t*  win   = reinterpret_cast<const uint8_t*>(win4 + 1);
    const uint32_t* win32 = reinterpret_cast<const uint32_t*>(win4 + 1);
    const int      lane = lane_id();
    const uint32_t k    = wave_id();  // this wave's sub-window (wave-uniform: its loops run on scalar registers)
    const uint64_t below = (1ull << lane) - 1ull;
    const uint64_t nunits = (uint64_t) nblocks * sg.nseg;
    for (uint64_t u = blockIdx.x; u < nunits; u += gridDim.x)
    {
        const uint32_t b    = (uint32_t) (u / sg.nseg);
        const uint32_t seg0 = (uint32_t) (u % sg.nseg) * sg.seg_bytes;
        const uint8_t* src  = in + in_base[b];
        const uint32_t size = in_size[b];
        if (sg.nseg > 1 && seg0 >= size)
            continue;  // no such segment (uniform over the workgroup)
        const uint32_t seg1 = sg.nseg > 1 ? min(size, seg0 + sg.seg_bytes) : size;
        uint8_t*       dst  = out + out_base[b];
        const uint64_t cap  = out_cap[b];
        // MAP: lane t < RD_NENT follows the chain entering the segment at offset t
        uint32_t me = threadIdx.x, mo = 0;
        if (!MAP && threadIdx.x == 0)
        {
            const uint2 st = sg.nseg > 1 ? sg.state[u] : make_uint2(0, 0);
            sh_E           = st.x;
            sh_O           = st.y;
        }
        // prefetch the segment's first window
        uint4 pf[2];
#pragma unroll
        for (int h = 0; h < 2; ++h)
        {
            const uint32_t t = threadIdx.x + h * RD_TPB;
            pf[h]            = t < RD_LOAD ? load16(src, size, seg0 + t * 16) : make_uint4(0, 0, 0, 0);
        }
        [[maybe_unused]] unsigned long long rt[4] = {0, 0, 0, 0}, rc = RT_NOW();
        for (uint32_t w0 = seg0; w0 < seg1; w0 += RD_WIN)
        {
            __syncthreads();  // previous window fully consumed
#pragma unroll
            for (int h = 0; h < 2; ++h)
            {
                const uint32_t t = threadIdx.x + h * RD_TPB;
                if (t < RD_LOAD)
                    win4[1 + t] = pf[h];
            }
            __syncthreads();
            // prefetch the next window while this one is decoded
            if (w0 + RD_WIN < seg1)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                {
                    const uint32_t t = threadIdx.x + h * RD_TPB;
                    pf[h]            = t < RD_LOAD ? load16(src, size, w0 + RD_WIN + t * 16) : make_uint4(0, 0, 0, 0);
                }

            // ---- 1. chain exits of every position of this wave's sub-window ----
            const uint32_t sb  = k * RD_SUB;
            const uint32_t rem = size - w0;
            const uint32_t len = rem > sb ? min(RD_SUB, rem - sb) : 0u;
            uint32_t       nx0[RD_PER], v[RD_PER];
#pragma unroll
            for (int m = 0; m < (int) RD_PER; ++m)
            {
                const uint32_t p = m * 64 + lane;
                const uint32_t c = win[sb + p];
                nx0[m]           = p + ctl_step(c);
                v[m]             = nx0[m] | ctl_prod(c) << PK_SH;
                if (p < len)
                    PK[k][p] = v[m];
            }
            wave_lds_sync();
#ifdef BRA_RLED_TIMING
            {
                const unsigned long long t = RT_NOW();
                rt[0] += t - rc;
                rc = t;
            }
#endif
            while (true)
            {
                bool     act = false;
                uint32_t nn[RD_PER];
#pragma unroll
                for (int m = 0; m < (int) RD_PER; ++m)
                {
                    const uint32_t p = m * 64 + lane, nx = v[m] & PK_POS;
                    nn[m]            = v[m];
                    if (p < len && nx < len)
                    {
                        nn[m] = (v[m] & ~PK_POS) + PK[k][nx];  // successor's successor, counts added
                        act   = true;
                    }
                }
                if (!__builtin_amdgcn_ballot_w64(act))
                    break;
                wave_lds_sync();
#pragma unroll
                for (int m = 0; m < (int) RD_PER; ++m)
                {
                    const uint32_t p = m * 64 + lane;
                    if (p < len && (v[m] & PK_POS) < len)
                    {
                        v[m]     = nn[m];
                        PK[k][p] = v[m];
                    }
                }
                wave_lds_sync();
            }
            __syncthreads();
#ifdef BRA_RLED_TIMING
            {
                const unsigned long long t = RT_NOW();
                rt[1] += t - rc;
                rc = t;
            }
#endif

            // ---- 2. entries and output offsets of the sub-windows ----
            if (MAP)
            {
                // every entry's chain through the 16 sub-windows
                if (threadIdx.x < RD_NENT)
                {
                    uint32_t e = me;
                    for (uint32_t q = 0; q < RD_WAVES; ++q)
                    {
                        const uint32_t qb = q * RD_SUB;
                        const uint32_t ql = rem > qb ? min(RD_SUB, rem - qb) : 0u;
                        if (e - qb < ql)
                        {
                            const uint32_t x = PK[q][e - qb];
                            mo += x >> PK_SH;
                            e = qb + (x & PK_POS);
                        }
                    }
                    me = e - RD_WIN;
                }
                continue;  // the loop head's barrier orders these reads before the next window's writes
            }
            if (threadIdx.x == 0)
            {
                uint32_t e = sh_E, o = sh_O;  // e: window offset of the next control
                for (uint32_t q = 0; q < RD_WAVES; ++q)
                {
                    const uint32_t qb = q * RD_SUB;
                    const uint32_t ql = rem > qb ? min(RD_SUB, rem - qb) : 0u;
                    sub_entry[q]      = e - qb;  // >= ql: the chain skips this sub-window (end of stream)
                    sub_out[q]        = o;
                    uint32_t t        = 0;
                    if (e - qb < ql)
                    {
                        const uint32_t x = PK[q][e - qb];
                        t                = x >> PK_SH;
                        e                = qb + (x & PK_POS);
                    }
                    sub_tot[q] = t;
                    o += t;
                }
                sh_E = e - RD_WIN;  // entry of the next window (exit offset past the stream end at the last one)
                sh_O = o;
            }
            __syncthreads();
#ifdef BRA_RLED_TIMING
            {
                const unsigned long long t = RT_NOW();
                rt[2] += t - rc;
                rc = t;
            }
#endif

            // ---- 3. walk the chain through this sub-window, compact it, write the output ----
            const uint32_t ent  = sub_entry[k];
            uint32_t       ncon = 0;
            if (ent < len)
            {
                const uint32_t sm_entry = PK[k][ent] >> PK_SH;
                wave_lds_sync();  // everyone read PK[k][ent] before the compaction overwrites it
                uint32_t e = ent;
#pragma unroll
                for (int m = 0; m < (int) RD_PER; ++m)
                {
                    uint64_t       on  = 0;
                    const uint32_t top = min((uint32_t) (m + 1) * 64u, len);
                    while (e < top)
                    {
                        const uint32_t l = e - m * 64;
                        on |= 1ull << l;
                        e = (uint32_t) __builtin_amdgcn_readlane((int) nx0[m], (int) l);
                    }
                    if ((on >> lane) & 1)
                    {
                        const uint32_t idx = ncon + (uint32_t) __popcll(on & below);
                        PK[k][idx]         = (m * 64 + lane) | (sm_entry - (v[m] >> PK_SH)) << PK_SH;  // position | output offset inside the sub-window's range
                    }
                    ncon += (uint32_t) __popcll(on);
                }
                wave_lds_sync();
            }
            if (lane == 0)
                sub_ncon[k] = ncon;
            __syncthreads();  // every sub-window's control list is compacted
            // Output bytes of the whole window, [sub_out[0], sh_O), 16 per thread per round over the
            // workgroup (a run-dense sub-window decodes to up to 64 KiB, a literal-dense one to about
            // 1 KiB: writing each sub-window's range with its own wave left the workgroup waiting for
            // its heaviest wave at the next barrier).  A thread's 16 bytes start in the last
            // sub-window holding output at or before them and may continue into the next ones.
            const uint32_t ow0 = sub_out[0], otot = sh_O - ow0;
            for (uint32_t r0 = 0; r0 < otot; r0 += RD_TPB * 16)
            {
                const uint32_t o0 = r0 + threadIdx.x * 16;  // relative to ow0
                if (o0 < otot)
                {
                    uint32_t kk = 0;
#pragma unroll
                    for (uint32_t q = 1; q < RD_WAVES; ++q)
                        if (sub_out[q] - ow0 <= o0 && sub_tot[q] > 0)
                            kk = q;
                    uint32_t base = sub_out[kk] - ow0, nk = sub_ncon[kk], tk = sub_tot[kk];
                    // last control of sub-window kk with offset <= o0 - base
                    uint32_t lo = 0, hi = nk - 1;
                    while (lo < hi)
                    {
                        const uint32_t mid = (lo + hi + 1) >> 1;
                        if ((PK[kk][mid] >> PK_SH) <= o0 - base)
                            lo = mid;
                        else
                            hi = mid - 1;
                    }
                    uint32_t idx = lo, d = PK[kk][idx] >> PK_SH, p = PK[kk][idx] & PK_POS;
                    uint32_t dn = idx + 1 < nk ? PK[kk][idx + 1] >> PK_SH : tk;
                    uint32_t wv[4] = {0, 0, 0, 0};
                    const uint32_t nb = min(16u, otot - o0);
                    // one piece per control covering part of the thread's 16 bytes: a run fills its
                    // bytes with one value, a literal copies a 16-byte unaligned LDS read (5 dwords
                    // + alignbyte) positioned so that byte j of it is output byte j; bytes outside
                    // [j, j + n) are kept by a bitfield insert
                    for (uint32_t j = 0; j < nb;)
                    {
                        uint32_t o = o0 + j - base;  // relative to sub-window kk's output
                        while (o >= dn)
                        {
                            if (idx + 1 < nk)
                            {
                                ++idx;
                                d  = dn;
                                p  = PK[kk][idx] & PK_POS;
                                dn = idx + 1 < nk ? PK[kk][idx + 1] >> PK_SH : tk;
                            }
                            else
                            {
                                // past sub-window kk's output: the next one holding output
                                do
                                    ++kk;
                                while (sub_tot[kk] == 0);
                                base = sub_out[kk] - ow0, nk = sub_ncon[kk], tk = sub_tot[kk];
                                o    = o0 + j - base;
                                idx = 0, d = 0, p = PK[kk][0] & PK_POS;
                                dn = nk > 1 ? PK[kk][1] >> PK_SH : tk;
                            }
                        }
                        const uint32_t at = kk * RD_SUB + p;
                        const uint32_t c  = win[at];
                        const uint32_t n  = min(dn - o, nb - j);
                        uint32_t       v[4];
                        if (c > 128u)
                        {
                            const uint32_t r = win[at + 1] * 0x01010101u;
                            v[0] = v[1] = v[2] = v[3] = r;
                        }
                        else
                        {
                            const int32_t  base4 = (int32_t) (at + 1 + (o - d)) - (int32_t) j;  // >= -15
                            const int32_t  a4    = (base4 >> 2);                               // floor
                            const uint32_t sh    = (uint32_t) base4 & 3u;
                            uint32_t       W[5];
#pragma unroll
                            for (int i = 0; i < 5; ++i)
                                W[i] = win32[a4 + i];
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                v[i] = __builtin_amdgcn_alignbyte(W[i + 1], W[i], sh);
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                        {
                            const int32_t  lo8 = min(max((int32_t) j - 4 * i, 0), 4), hi8 = min(max((int32_t) (j + n) - 4 * i, 0), 4);
                            const uint32_t mh  = hi8 >= 4 ? 0xFFFFFFFFu : (1u << (8 * hi8)) - 1u;
                            const uint32_t ml  = lo8 >= 4 ? 0xFFFFFFFFu : (1u << (8 * lo8)) - 1u;
                            const uint32_t m   = mh & ~ml;
                            wv[i]              = (v[i] & m) | (wv[i] & ~m);
                        }
                        j += n;
                    }
                    const uint64_t a = (uint64_t) ow0 + o0;  // block output offset
                    uint8_t*       q = dst + a;
                    if (nb == 16 && a + 16 <= cap)  // one (unaligned) 16-byte store: the output offsets have any alignment
                        *reinterpret_cast<u128_u*>(q) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                    else
                        for (uint32_t j = 0; j < nb; ++j)
                            if (a + j < cap)
                                q[j] = (uint8_t) (wv[j >> 2] >> (8 * (j & 3)));
                }
            }
#ifdef BRA_RLED_TIMING
            {
                const unsigned long long t = RT_NOW();
                rt[3] += t - rc;
                rc = t;
            }
#endif
        }
#ifdef BRA_RLED_TIMING
        if (threadIdx.x == 0)
            for (int i = 0; i < 4; ++i)
                atomicAdd(&g_rled_t[i], rt[i]);
#endif
        __syncthreads();
        if (MAP)
        {
            if (threadIdx.x < RD_NENT)
                sg.map[u * RD_NENT + threadIdx.x] = make_uint2(me, mo);
        }
        else if (sg.nseg == 1 && threadIdx.x == 0)
        {
            // the chain must end exactly at the end of the stream (sh_E = its overshoot past the
            // window holding the stream end, measured from that window's end: recompute it)
            const uint32_t last_w0 = size ? ((size - 1) / RD_WIN) * RD_WIN : 0u;
            const uint32_t over    = (sh_E + RD_WIN) - (size - last_w0);  // exit position minus stream length
            out_size[b]            = (size == 0 || over != 0) ? 0u : sh_O;
        }
        __syncthreads();
    }
}

// One lane per block: chain the segments through their entry maps (a segment ends with a whole
// window, so the exit offset past it is the next segment's entry, in [0, 128] for a stream that
// continues), record each segment's entry and output offset, and the decoded size (0 unless the
// chain ends exactly at the end of the stream, as in k_rled).
__global__ void k_rled_link(const uint32_t* __restrict__ in_size, uint32_t nblocks, uint32_t* __restrict__ out_size, RledSeg sg)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks)
        return;
    const uint32_t size = in_size[b];
    if (size == 0)
    {
        out_size[b] = 0;
        return;
    }
    const uint32_t nj = (size - 1) / sg.seg_bytes + 1;  // <= nseg (the host sized nseg for the largest stream)
    uint32_t       e = 0, o = 0;
    bool           ok = true;
    for (uint32_t j = 0; j < nj; ++j)
    {
        const uint64_t u = (uint64_t) b * sg.nseg + j;
        if (e >= RD_NENT)
        {
            ok = false;  // only a malformed stream's chain can skip past a segment's first 129 bytes
            e  = 0;
        }
        sg.state[u]   = make_uint2(e, o);
        const uint2 m = sg.map[u * RD_NENT + e];
        o += m.y;
        e = m.x;
    }
    const uint32_t last_w0 = ((size - 1) / RD_WIN) * RD_WIN;
    const uint32_t over    = (e + RD_WIN) - (size - last_w0);
    out_size[b]            = (!ok || over != 0) ? 0u : o;
}

}  // namespace

bool rle_decode_device(RleWorkspace& w, const uint32_t* h_in_size, const uint8_t* d_in, const uint64_t* d_in_base, const uint32_t* d_in_size,
                       uint32_t nblocks, uint8_t* d_out, const uint64_t* d_out_base, const uint64_t* d_out_cap, uint32_t* d_out_size,
                       hipStream_t s)
{
    BRA_PROF(P_DEC_RLED, s);
    // segments (about RD_TARGET_WG workgroups over the batch) only when the blocks alone would leave
    // at least half of the 256 CUs idle: the map pass costs about as much as the decode itself
    // (256 x 1 MiB text: 2.13 ms whole blocks, 3.26 ms in segments; 32 x 8 MiB sym16: 21.2 -> 4.0 ms)
    constexpr uint32_t RD_TARGET_WG = 512, RD_SEG_MAX_BLOCKS = 128;
    uint32_t           maxsz        = 0;
    for (uint32_t b = 0; h_in_size && b < nblocks; ++b)
        maxsz = std::max(maxsz, h_in_size[b]);
    RledSeg sg{1, 0, nullptr, nullptr};
    if (h_in_size && nblocks <= RD_SEG_MAX_BLOCKS && maxsz > 2 * RD_WIN)
    {
        const uint32_t want = div_up(RD_TARGET_WG, nblocks);
        const uint32_t wins = div_up(maxsz, RD_WIN);
        const uint32_t per  = std::max(4u, div_up(wins, std::min(want, wins)));  // windows per segment (>= 64 KiB: short link chains)
        sg.seg_bytes        = per * RD_WIN;
        sg.nseg             = div_up(maxsz, sg.seg_bytes);
    }
    if (sg.nseg > 1)
    {
        const uint64_t units = (uint64_t) nblocks * sg.nseg;
        if (!w.reserve_decode(units * (RD_NENT + 1) * sizeof(uint2)))
            return false;
        sg.map   = static_cast<uint2*>(w.dmap);
        sg.state = sg.map + units * RD_NENT;
        const uint32_t g = (uint32_t) std::min<uint64_t>(units, 65535);
        hipLaunchKernelGGL(k_rled<true>, dim3(g), dim3(RD_TPB), 0, s, d_in, d_in_base, d_in_size, nblocks, d_out, d_out_base, d_out_cap,
                           d_out_size, sg);
        hipLaunchKernelGGL(k_rled_link, dim3(div_up(nblocks, 64u)), dim3(64), 0, s, d_in_size, nblocks, d_out_size, sg);
        hipLaunchKernelGGL(k_rled<false>, dim3(g), dim3(RD_TPB), 0, s, d_in, d_in_base, d_in_size, nblocks, d_out, d_out_base, d_out_cap,
                           d_out_size, sg);
    }
    else
        hipLaunchKernelGGL(k_rled<false>, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(RD_TPB), 0, s, d_in, d_in_base, d_in_size, nblocks,
                           d_out, d_out_base, d_out_cap, d_out_size, sg);
    BRA_HIP_CHECK(hipGetLastError());
#ifdef BRA_RLED_TIMING
    {
        unsigned long long t[4] = {0, 0, 0, 0}, z[4] = {0, 0, 0, 0};
        if (hipStreamSynchronize(s) == hipSuccess && hipMemcpyFromSymbol(t, HIP_SYMBOL(g_rled_t), sizeof t) == hipSuccess)
            fprintf(stderr, "rled clocks (wave 0, summed): load+ptr-init %llu  pointer-jumping %llu  entries %llu  walk+write %llu\n", t[0], t[1], t[2],
                    t[3]);
        (void) hipMemcpyToSymbol(HIP_SYMBOL(g_rled_t), z, sizeof z);
    }
#endif
    return true;
}

}  // namespace bra
