// bra_hip_common.h -- shared host/device helpers for the gfx950 block-codec kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define BRA_HIP_CHECK(expr)                                                                              \
    do                                                                                                   \
    {                                                                                                    \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess)                                                                            \
        {                                                                                                \
            bra_hip_report("HIP error %s at %s:%d: %s", hipGetErrorString(_e), __FILE__, __LINE__, #expr); \
            return false;                                                                                \
        }                                                                                                \
    } while (0)

// Error sink: forwards to the reference's bra_log_error when lib_bra is linked in, else stderr.
void bra_hip_report(const char* fmt, ...);

// Device-side range checks for debugging (make EXTRA=-DBRA_DEBUG): print the violation and let
// the caller sanitise the value; compiled out otherwise.
#ifdef BRA_DEBUG
#define BRA_DCHECK(cond, ...)                           \
    (__builtin_expect(!(cond), 0) ? (printf("[bra dcheck] %s:%d ", __FILE__, __LINE__), printf(__VA_ARGS__), printf("\n"), false) : true)
#else
#define BRA_DCHECK(cond, ...) true
#endif

namespace bra {

constexpr int WAVE = 64;

// (Re)allocate device buffer p for `elems` elements of T, dropping its old contents.  On failure p
// is null and false is returned; callers zero their capacity field BEFORE calling and set it only
// after every allocation of the group succeeded, so a failed grow never leaves a stale capacity
// next to a null pointer (a later, smaller request would otherwise launch kernels on null).
template <typename T>
inline bool dev_alloc(T*& p, uint64_t elems)
{
    (void) hipFree(p);
    p            = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), (size_t) (elems ? elems : 1) * sizeof(T));
    if (e != hipSuccess)
    {
        p = nullptr;
        (void) hipGetLastError();
        bra_hip_report("device allocation of %llu bytes failed: %s", (unsigned long long) (elems * sizeof(T)), hipGetErrorString(e));
        return false;
    }
    return true;
}

inline bool dev_alloc_bytes(void*& p, uint64_t bytes)
{
    uint8_t*   q  = static_cast<uint8_t*>(p);
    const bool ok = dev_alloc(q, bytes);
    p             = q;
    return ok;
}

// ---------------------------------------------------------------------------------------------
// Batch geometry: a batch is `nblocks` independent blocks laid out back to back in HBM.
// ---------------------------------------------------------------------------------------------
struct BlockDesc
{
    uint64_t off;  // byte offset of the block in the batch (== slot offset of its rotations)
    uint32_t len;  // block length n (1 <= n < 2^24)
    uint32_t pad;
};

// ---------------------------------------------------------------------------------------------
// Wave-level helpers (wave64).  Elements are distributed 4 per lane: element e = 4*lane + r.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// The wave's index in its workgroup, wave-uniform to the compiler: threadIdx.x >> 6 is not (the
// compiler treats it as per-lane), so loops and branches on it ran under exec masks with VALU
// compares and readfirstlanes; through readfirstlane they run on scalar registers.  Round 6, one
// box, two A/B pairs: wave jobs 1.82 -> 1.73 ms (k_jobs 73 -> 55 VGPRs), MTF last occurrences
// 0.139 -> 0.124 ms, the RLE decode's chain walk a 5-instruction scalar loop (it was 12 with
// exec-mask juggling and s_nops).
__device__ __forceinline__ uint32_t wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m)
{
    uint32_t lo = (uint32_t) v, hi = (uint32_t) (v >> 32);
    lo          = __shfl_xor(lo, m, WAVE);
    hi          = __shfl_xor(hi, m, WAVE);
    return ((uint64_t) hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d)
{
    uint32_t lo = (uint32_t) v, hi = (uint32_t) (v >> 32);
    lo          = __shfl_up(lo, d, WAVE);
    hi          = __shfl_up(hi, d, WAVE);
    return ((uint64_t) hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_down64(uint64_t v, int d)
{
    uint32_t lo = (uint32_t) v, hi = (uint32_t) (v >> 32);
    lo          = __shfl_down(lo, d, WAVE);
    hi          = __shfl_down(hi, d, WAVE);
    return ((uint64_t) hi << 32) | lo;
}

// (key, val) lexicographic "greater than".
__device__ __forceinline__ bool kv_gt(uint64_t ka, uint32_t va, uint64_t kb, uint32_t vb)
{
    return ka > kb || (ka == kb && va > vb);
}

// Bitonic sort of P (4..256, power of two) elements held 4 per lane, ascending by (key, val).
// Lanes >= P/4 hold padding and take part only in their own (ignored) sub-network.
__device__ __forceinline__ void wave_bitonic_sort4(uint64_t (&k)[4], uint32_t (&v)[4], int P)
{
    const int lane = lane_id();
    for (int size = 2; size <= P; size <<= 1)
    {
        for (int j = size >> 1; j > 0; j >>= 1)
        {
            if (j >= 4)
            {
                const int lm = j >> 2;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                {
                    const int      e    = lane * 4 + r;
                    const uint64_t ok   = shfl_xor64(k[r], lm);
                    const uint32_t ov   = __shfl_xor(v[r], lm, WAVE);
                    const bool     up   = (e & size) == 0;
                    const bool     low  = (e & j) == 0;
                    const bool     gt   = kv_gt(k[r], v[r], ok, ov);
                    // lower element keeps min when ascending, max when descending
                    const bool     take = (low == up) ? gt : !gt;
                    if (take && !(k[r] == ok && v[r] == ov))
                    {
                        k[r] = ok;
                        v[r] = ov;
                    }
                }
            }
            else
            {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                {
                    const int p = r ^ j;
                    if (p > r)
                    {
                        const int  e  = lane * 4 + r;
                        const bool up = (e & size) == 0;
                        const bool gt = kv_gt(k[r], v[r], k[p], v[p]);
                        if (gt == up)
                        {
                            uint64_t tk = k[r];
                            k[r]        = k[p];
                            k[p]        = tk;
                            uint32_t tv = v[r];
                            v[r]        = v[p];
                            v[p]        = tv;
                        }
                    }
                }
            }
        }
    }
}

// Inclusive max-scan over 256 elements (4 per lane) in element order.
// ---- wave / workgroup scans on one dword per thread (DPP inside rows of 16, row totals by
// readlane; no LDS inside a wave) ----
struct OpMax
{
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return max(a, b); }
};
struct OpMin
{
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return min(a, b); }
};
struct OpAdd
{
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};
struct OpOr
{
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; }
};

// Inclusive scan over the lanes of a wave in increasing (FWD) or decreasing lane order.
// Inclusive scan over the lanes of a wave in increasing (FWD) or decreasing lane order; with `ex`,
// also the exclusive value (the scan of the lanes before this one in scan order, id for the first).
// DPP row shifts inside rows of 16 lanes, row totals by readlane (DPP wave shifts do not cross
// rows on gfx950).
template <bool FWD, typename Op>
__device__ __forceinline__ uint32_t wave_scan(uint32_t x, uint32_t id, Op op, uint32_t* ex = nullptr)
{
    const uint32_t row = (uint32_t) lane_id() >> 4;
    if (FWD)
    {
        x = op(x, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x111, 0xf, 0xf, false));  // row_shr:1
        x = op(x, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x112, 0xf, 0xf, false));  // row_shr:2
        x = op(x, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x114, 0xf, 0xf, false));  // row_shr:4
        x = op(x, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x118, 0xf, 0xf, false));  // row_shr:8
        const uint32_t t0 = __builtin_amdgcn_readlane(x, 15), t1 = __builtin_amdgcn_readlane(x, 31), t2 = __builtin_amdgcn_readlane(x, 47);
        const uint32_t c1 = t0, c2 = op(t0, t1), c3 = op(c2, t2);
        const uint32_t carry = row == 0 ? id : row == 1 ? c1 : row == 2 ? c2 : c3;
        if (ex)
            *ex = op(carry, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x111, 0xf, 0xf, false));
        return op(x, carry);
    }
    x = op(x, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x101, 0xf, 0xf, false));  // row_shl:1
    x = op(x, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x102, 0xf, 0xf, false));  // row_shl:2
    x = op(x, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x104, 0xf, 0xf, false));  // row_shl:4
    x = op(x, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x108, 0xf, 0xf, false));  // row_shl:8
    const uint32_t t1 = __builtin_amdgcn_readlane(x, 16), t2 = __builtin_amdgcn_readlane(x, 32), t3 = __builtin_amdgcn_readlane(x, 48);
    const uint32_t c2 = t3, c1 = op(t2, t3), c0 = op(t1, c1);
    const uint32_t carry = row == 3 ? id : row == 2 ? c2 : row == 1 ? c1 : c0;
    if (ex)
        *ex = op(carry, (uint32_t) __builtin_amdgcn_update_dpp((int) id, (int) x, 0x101, 0xf, 0xf, false));
    return op(x, carry);
}

__device__ __forceinline__ void wave_max_scan4(uint32_t (&x)[4])
{
    x[1]              = max(x[1], x[0]);
    x[2]              = max(x[2], x[1]);
    x[3]              = max(x[3], x[2]);
    uint32_t ex;
    wave_scan<true>(x[3], 0u, OpMax(), &ex);
#pragma unroll
    for (int r = 0; r < 4; ++r)
        x[r] = max(x[r], ex);
}

// XCD-major tile ranges: workgroup w runs on XCD w % 8 and walks the XCD's contiguous eighth of
// the tile list, so neighbouring tiles (whose outputs share boundary lines) run on one XCD and
// meet in its L2.  Plain round robin when the grid is not a multiple of 8.
struct XcdTiles
{
    uint32_t t, end, step;
};
__device__ __forceinline__ XcdTiles xcd_tiles(uint32_t ntiles)
{
    if (gridDim.x < 8 || (gridDim.x & 7) != 0)
        return XcdTiles{blockIdx.x, ntiles, gridDim.x};
    const uint32_t per = (ntiles + 7u) / 8u, t0 = (blockIdx.x & 7u) * per;
    return XcdTiles{t0 + (blockIdx.x >> 3), min(ntiles, t0 + per), gridDim.x >> 3};
}
__host__ __device__ inline uint32_t xcd_grid(uint32_t g) { return g >= 8 ? g & ~7u : g; }

// Value of x held by lane (lane ^ LM), LM in {1, 2, 4, 8, 16, 32}, without going through LDS:
// DPP quad permutes / row rotate inside a row of 16 (one instruction each), xor 4 as two row shifts
// writing complementary bank masks (lanes with bit 2 clear take lane + 4, the others lane - 4), and
// permlane swaps across rows.
template <int LM>
__device__ __forceinline__ uint32_t xlane(uint32_t x)
{
    if constexpr (LM == 1)
        return (uint32_t) __builtin_amdgcn_mov_dpp((int) x, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    else if constexpr (LM == 2)
        return (uint32_t) __builtin_amdgcn_mov_dpp((int) x, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    else if constexpr (LM == 4)
    {
        const int up = __builtin_amdgcn_mov_dpp((int) x, 0x104, 0xF, 0x5, false);             // row_shl:4 into banks 0, 2
        return (uint32_t) __builtin_amdgcn_update_dpp(up, (int) x, 0x114, 0xF, 0xA, false);  // row_shr:4 into banks 1, 3
    }
    else if constexpr (LM == 8)
        return (uint32_t) __builtin_amdgcn_mov_dpp((int) x, 0x128, 0xF, 0xF, true);  // row_ror:8
    else if constexpr (LM == 16)
    {
        const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane_id() & 16) ? p[0] : p[1];
    }
    else
    {
        static_assert(LM == 32, "lane distance");
        const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane_id() & 32) ? p[0] : p[1];
    }
}

// Every compare-exchange string writes VCC and, through its s_xnor_b64, SCC: both are declared
// clobbered.  (Without "scc" the compiler kept a lane-mask select's SCC live across the string and
// the s_cselect after it picked the mask from the xnor's result instead -- a network stage with the
// inverted direction whenever the xnor came out zero, i.e. for some key sets only: the intermittent
// wrong BWT blocks, found by replaying a failing job sort phase by phase, scripts/rerun_jobs.py.)
// 128-bit keys as four dwords (k0 lowest).  k > o is the borrow out of the 128-bit subtraction
// o - k: four chained VALU subtractions into VCC, so a compare-exchange is 4 subtractions, one SALU
// xnor with a lane mask and 4 selects (the C++ form compiles to three 64-bit compares, SALU
// and/or and the selects).  Dword operands keep the compiler from pairing registers.
// Compare-exchange with the partner's key o: the lanes whose (k > o) equals their bit of
// `keep_min` take o.
__device__ __forceinline__ void cx128(uint32_t& k0, uint32_t& k1, uint32_t& k2, uint32_t& k3, uint32_t o0, uint32_t o1, uint32_t o2,
                                      uint32_t o3, uint64_t keep_min)
{
    uint32_t t;
    asm volatile(
        "v_sub_co_u32 %[t], vcc, %[o0], %[k0]\n\t"
        "v_subb_co_u32 %[t], vcc, %[o1], %[k1], vcc\n\t"
        "v_subb_co_u32 %[t], vcc, %[o2], %[k2], vcc\n\t"
        "v_subb_co_u32 %[t], vcc, %[o3], %[k3], vcc\n\t"
        "s_xnor_b64 vcc, vcc, %[km]\n\t"
        "v_cndmask_b32 %[k0], %[k0], %[o0], vcc\n\t"
        "v_cndmask_b32 %[k1], %[k1], %[o1], vcc\n\t"
        "v_cndmask_b32 %[k2], %[k2], %[o2], vcc\n\t"
        "v_cndmask_b32 %[k3], %[k3], %[o3], vcc"
        : [t] "=&v"(t), [k0] "+v"(k0), [k1] "+v"(k1), [k2] "+v"(k2), [k3] "+v"(k3)
        : [o0] "v"(o0), [o1] "v"(o1), [o2] "v"(o2), [o3] "v"(o3), [km] "s"(keep_min)
        : "vcc", "scc");
}

// In-lane compare-exchange of keys a and b: afterwards a < b in the lanes set in `asc`, a > b in
// the others (the selects write fresh registers, so no copies).
__device__ __forceinline__ void cx128_pair(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3, uint32_t& b0, uint32_t& b1, uint32_t& b2,
                                           uint32_t& b3, uint64_t asc)
{
    uint32_t t, n0, n1, n2, n3, m0, m1, m2, m3;
    asm volatile(
        "v_sub_co_u32 %[t], vcc, %[b0], %[a0]\n\t"
        "v_subb_co_u32 %[t], vcc, %[b1], %[a1], vcc\n\t"
        "v_subb_co_u32 %[t], vcc, %[b2], %[a2], vcc\n\t"
        "v_subb_co_u32 %[t], vcc, %[b3], %[a3], vcc\n\t"
        "s_xnor_b64 vcc, vcc, %[asc]\n\t"
        "v_cndmask_b32 %[n0], %[a0], %[b0], vcc\n\t"
        "v_cndmask_b32 %[m0], %[b0], %[a0], vcc\n\t"
        "v_cndmask_b32 %[n1], %[a1], %[b1], vcc\n\t"
        "v_cndmask_b32 %[m1], %[b1], %[a1], vcc\n\t"
        "v_cndmask_b32 %[n2], %[a2], %[b2], vcc\n\t"
        "v_cndmask_b32 %[m2], %[b2], %[a2], vcc\n\t"
        "v_cndmask_b32 %[n3], %[a3], %[b3], vcc\n\t"
        "v_cndmask_b32 %[m3], %[b3], %[a3], vcc"
        : [t] "=&v"(t), [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2), [n3] "=&v"(n3), [m0] "=&v"(m0), [m1] "=&v"(m1), [m2] "=&v"(m2),
          [m3] "=&v"(m3)
        : [a0] "v"(a0), [a1] "v"(a1), [a2] "v"(a2), [a3] "v"(a3), [b0] "v"(b0), [b1] "v"(b1), [b2] "v"(b2), [b3] "v"(b3), [asc] "s"(asc)
        : "vcc", "scc");
    a0 = n0, a1 = n1, a2 = n2, a3 = n3;
    b0 = m0, b1 = m1, b2 = m2, b3 = m3;
}

// 96-bit keys as three dwords (k0 lowest): the same compare-exchange with three subtractions and
// three selects (the job sort network; a 96-bit key holds 11 rotation bytes after the slot bits).
__device__ __forceinline__ void cx96(uint32_t& k0, uint32_t& k1, uint32_t& k2, uint32_t o0, uint32_t o1, uint32_t o2, uint64_t keep_min)
{
    uint32_t t;
    asm volatile(
        "v_sub_co_u32 %[t], vcc, %[o0], %[k0]\n\t"
        "v_subb_co_u32 %[t], vcc, %[o1], %[k1], vcc\n\t"
        "v_subb_co_u32 %[t], vcc, %[o2], %[k2], vcc\n\t"
        "s_xnor_b64 vcc, vcc, %[km]\n\t"
        "v_cndmask_b32 %[k0], %[k0], %[o0], vcc\n\t"
        "v_cndmask_b32 %[k1], %[k1], %[o1], vcc\n\t"
        "v_cndmask_b32 %[k2], %[k2], %[o2], vcc"
        : [t] "=&v"(t), [k0] "+v"(k0), [k1] "+v"(k1), [k2] "+v"(k2)
        : [o0] "v"(o0), [o1] "v"(o1), [o2] "v"(o2), [km] "s"(keep_min)
        : "vcc", "scc");
}

__device__ __forceinline__ void cx96_pair(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& b0, uint32_t& b1, uint32_t& b2, uint64_t asc)
{
    uint32_t t, n0, n1, n2, m0, m1, m2;
    asm volatile(
        "v_sub_co_u32 %[t], vcc, %[b0], %[a0]\n\t"
        "v_subb_co_u32 %[t], vcc, %[b1], %[a1], vcc\n\t"
        "v_subb_co_u32 %[t], vcc, %[b2], %[a2], vcc\n\t"
        "s_xnor_b64 vcc, vcc, %[asc]\n\t"
        "v_cndmask_b32 %[n0], %[a0], %[b0], vcc\n\t"
        "v_cndmask_b32 %[m0], %[b0], %[a0], vcc\n\t"
        "v_cndmask_b32 %[n1], %[a1], %[b1], vcc\n\t"
        "v_cndmask_b32 %[m1], %[b1], %[a1], vcc\n\t"
        "v_cndmask_b32 %[n2], %[a2], %[b2], vcc\n\t"
        "v_cndmask_b32 %[m2], %[b2], %[a2], vcc"
        : [t] "=&v"(t), [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2), [m0] "=&v"(m0), [m1] "=&v"(m1), [m2] "=&v"(m2)
        : [a0] "v"(a0), [a1] "v"(a1), [a2] "v"(a2), [b0] "v"(b0), [b1] "v"(b1), [b2] "v"(b2), [asc] "s"(asc)
        : "vcc", "scc");
    a0 = n0, a1 = n1, a2 = n2;
    b0 = m0, b1 = m1, b2 = m2;
}

// 64-bit keys as two dwords (k0 lowest): the job sort network's keys (the rotation's packed bits
// above the slot bits).  Two subtractions, one xnor, two selects.
__device__ __forceinline__ void cx64(uint32_t& k0, uint32_t& k1, uint32_t o0, uint32_t o1, uint64_t keep_min)
{
    uint32_t t;
    asm volatile(
        "v_sub_co_u32 %[t], vcc, %[o0], %[k0]\n\t"
        "v_subb_co_u32 %[t], vcc, %[o1], %[k1], vcc\n\t"
        "s_xnor_b64 vcc, vcc, %[km]\n\t"
        "v_cndmask_b32 %[k0], %[k0], %[o0], vcc\n\t"
        "v_cndmask_b32 %[k1], %[k1], %[o1], vcc"
        : [t] "=&v"(t), [k0] "+v"(k0), [k1] "+v"(k1)
        : [o0] "v"(o0), [o1] "v"(o1), [km] "s"(keep_min)
        : "vcc", "scc");
}

__device__ __forceinline__ void cx64_pair(uint32_t& a0, uint32_t& a1, uint32_t& b0, uint32_t& b1, uint64_t asc)
{
    uint32_t t, n0, n1, m0, m1;
    asm volatile(
        "v_sub_co_u32 %[t], vcc, %[b0], %[a0]\n\t"
        "v_subb_co_u32 %[t], vcc, %[b1], %[a1], vcc\n\t"
        "s_xnor_b64 vcc, vcc, %[asc]\n\t"
        "v_cndmask_b32 %[n0], %[a0], %[b0], vcc\n\t"
        "v_cndmask_b32 %[m0], %[b0], %[a0], vcc\n\t"
        "v_cndmask_b32 %[n1], %[a1], %[b1], vcc\n\t"
        "v_cndmask_b32 %[m1], %[b1], %[a1], vcc"
        : [t] "=&v"(t), [n0] "=&v"(n0), [n1] "=&v"(n1), [m0] "=&v"(m0), [m1] "=&v"(m1)
        : [a0] "v"(a0), [a1] "v"(a1), [b0] "v"(b0), [b1] "v"(b1), [asc] "s"(asc)
        : "vcc", "scc");
    a0 = n0, a1 = n1;
    b0 = m0, b1 = m1;
}

// (Folding the lane exchange into the compare-exchange as DPP source operands -- v_sub_co / v_subb_co /
// v_cndmask with a DPP src0, 4 VALU instead of 6 -- is correct with the scc clobber (round 3's wrong
// sorts with it were the missing clobber) but measured equal in round 4: 1.889 vs 1.893 ms wave
// jobs, 3.25 ms workgroup jobs either way; the separate DPP moves stay.)
template <int LM>
__device__ __forceinline__ uint64_t xlane64(uint64_t x)
{
    return ((uint64_t) xlane<LM>((uint32_t) (x >> 32)) << 32) | xlane<LM>((uint32_t) x);
}

// Exclusive sum over 256 elements (4 per lane, element = lane * 4 + r); *total = sum of all.
__device__ __forceinline__ void wave_excl_sum4(const uint32_t (&x)[4], uint32_t (&ex)[4], uint32_t* total = nullptr)
{
    const uint32_t l1 = x[0], l2 = l1 + x[1], l3 = l2 + x[2], l4 = l3 + x[3];
    const uint32_t agg = wave_scan<true>(l4, 0u, OpAdd());
    if (total)
        *total = __builtin_amdgcn_readlane(agg, WAVE - 1);
    const uint32_t pre = agg - l4;
    ex[0]              = pre;
    ex[1]              = pre + l1;
    ex[2]              = pre + l2;
    ex[3]              = pre + l3;
}

// Exclusive max-scan over 256 elements (4 per lane); 0 for the first element.
__device__ __forceinline__ void wave_excl_max4(const uint32_t (&x)[4], uint32_t (&ex)[4])
{
    uint32_t inc[4] = {x[0], x[1], x[2], x[3]};
    inc[1]          = max(inc[1], inc[0]);
    inc[2]          = max(inc[2], inc[1]);
    inc[3]          = max(inc[3], inc[2]);
    uint32_t prev;
    wave_scan<true>(inc[3], 0u, OpMax(), &prev);
#pragma unroll
    for (int r = 0; r < 3; ++r)
        inc[r] = max(inc[r], prev);
    ex[0] = prev;
    ex[1]               = inc[0];
    ex[2]               = inc[1];
    ex[3]               = inc[2];
}

// Inclusive min-scan over 256 elements (4 per lane) in REVERSE element order.
__device__ __forceinline__ void wave_min_rscan4(uint32_t (&x)[4])
{
    x[2]              = min(x[2], x[3]);
    x[1]              = min(x[1], x[2]);
    x[0]              = min(x[0], x[1]);
    uint32_t ex;
    wave_scan<false>(x[0], 0xFFFFFFFFu, OpMin(), &ex);
#pragma unroll
    for (int r = 0; r < 4; ++r)
        x[r] = min(x[r], ex);
}

// Block-wide exclusive sum over 256 threads (one value per thread).  `tmp` >= 8 words of LDS.
__device__ __forceinline__ uint32_t block256_exclusive_sum(uint32_t v, uint32_t* tmp, uint32_t* total = nullptr)
{
    const int      lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t x    = wave_scan<true>(v, 0u, OpAdd());
    if (lane == WAVE - 1)
        tmp[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int i = 0; i < 4; ++i)
    {
        if (i < w)
            pre += tmp[i];
        tot += tmp[i];
    }
    __syncthreads();
    if (total)
        *total = tot;
    return pre + x - v;
}

__device__ __forceinline__ uint64_t block256_exclusive_sum64(uint64_t v, uint64_t* tmp, uint64_t* total = nullptr)
{
    const int lane = lane_id(), w = threadIdx.x >> 6;
    uint64_t  x    = v;
    for (int d = 1; d < WAVE; d <<= 1)
    {
        uint64_t o = shfl_up64(x, d);
        if (lane >= d)
            x += o;
    }
    if (lane == WAVE - 1)
        tmp[w] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (int i = 0; i < 4; ++i)
    {
        if (i < w)
            pre += tmp[i];
        tot += tmp[i];
    }
    __syncthreads();
    if (total)
        *total = tot;
    return pre + x - v;
}

// 8 cyclic bytes of a block starting at `start` (< n), big-endian (first byte most significant).
// Non-wrapping reads use two naturally aligned 8-byte loads: each aligned word holds at least one
// in-range byte, so the read never leaves the pages of the buffer.
__device__ __forceinline__ uint64_t load_key8(const uint8_t* __restrict__ blk, uint32_t n, uint32_t start)
{
    if (start + 8u <= n)
    {
        const uintptr_t a  = (uintptr_t) (blk + start);
        const uint64_t* p  = (const uint64_t*) (a & ~(uintptr_t) 7);
        const unsigned  sh = (unsigned) (a & 7) * 8u;
        uint64_t        w  = p[0] >> sh;
        if (sh)
            w |= p[1] << (64u - sh);
        return __builtin_bswap64(w);
    }
    uint64_t k = 0;
    uint32_t q = start;
    for (int i = 0; i < 8; ++i)
    {
        k = (k << 8) | blk[q];
        q = (q + 1 == n) ? 0 : q + 1;
    }
    return k;
}

__host__ __device__ __forceinline__ uint32_t div_up(uint64_t a, uint32_t b) { return (uint32_t) ((a + b - 1) / b); }

}  // namespace bra
