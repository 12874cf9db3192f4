// rle_tile.h -- per-thread PackBits classification and output of one RLE tile (rle.hip).
//
// A thread holds PT = 16 consecutive positions of a 4 KiB tile.  Which positions are covered by
// run blocks, which start one and which carry a literal block's control byte follows from the
// maximal runs and literal gaps (rle.hip header; reference src/encoders/bra_rle.c:60-120).  A
// run or gap that starts and ends inside the thread is shorter than 128, so it has its block
// start / control byte at its first position and nothing else: those are found for all 16
// positions at once with mask arithmetic; only the thread's first and last run and its first gap,
// which may continue from or into other threads and tiles, take per-segment arithmetic.  (The
// per-position form recomputed a run's extent at every position: 96 lane instructions per input
// byte, the RLE kernels' bound.)
//
// Plain integer code on 32-bit masks, compiled for the device by rle.hip and for the host by the
// CPU check tests/cpp/rle_tile_check.cpp, which compares whole blocks with the oracle encoder.
#pragma once
#include <cstdint>

#ifdef __HIPCC__
#define BRA_RT_HD __host__ __device__ __forceinline__
#else
#define BRA_RT_HD inline
#endif

namespace bra {
namespace rle_tile {

constexpr int PT = 16;  // positions per thread

BRA_RT_HD uint32_t hi_bit(uint32_t m) { return 31u - (uint32_t) __builtin_clz(m); }  // m != 0
BRA_RT_HD uint32_t lo_bit(uint32_t m) { return (uint32_t) __builtin_ctz(m); }        // m != 0
BRA_RT_HD uint32_t popc(uint32_t m) { return (uint32_t) __builtin_popcount(m); }
BRA_RT_HD uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
BRA_RT_HD uint32_t below(uint32_t i) { return (1u << i) - 1u; }  // i <= 16

BRA_RT_HD uint32_t byte_at(const uint32_t (&w)[4], int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; }

// Bit i set iff byte i differs from byte i-1 (bit 0: from `prev`), for the PT bytes of w.
BRA_RT_HD uint32_t diff_mask(const uint32_t (&w)[4], uint32_t prev)
{
    uint32_t m = 0, carry = prev & 0xFFu;
#pragma unroll
    for (int d = 0; d < 4; ++d)
    {
        const uint32_t z  = w[d] ^ ((w[d] << 8) | carry);                          // byte j: x[j] ^ x[j-1]
        const uint32_t nz = (((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;  // bit 7 of byte j: nonzero
        m |= ((((nz >> 7) * 0x01020408u) >> 24) & 0xFu) << (4 * d);
        carry = w[d] >> 24;
    }
    return m;
}

// Run classification of a thread's positions: nl = covered by run blocks, rs = run-block starts;
// the block length at a start in the thread's first / last segment (r0 / r1: that start's bit)
// is c0 / c1, anywhere else the length of its (inner, whole) run.
struct RunCls
{
    uint32_t nl, rs, r0, r1, c0, c1;
};

// Positions [lo, hi) of one maximal run of length L; k = position inside the run at lo.
// A position is covered iff L >= 3 and k < L - cut (cut: 1 or 2 tail bytes become literals);
// blocks start at k = 0 mod 128 and are min(128, L - k) long.
BRA_RT_HD void seg_cls(uint32_t lo, uint32_t hi, uint32_t k, uint32_t L, uint32_t& nl, uint32_t& rs, uint32_t& clen)
{
    const uint32_t tail = L & 127u, cut = tail < 3 ? tail : 0u;
    nl = rs = clen = 0;
    if (L < 3 || k >= L - cut)
        return;
    const uint32_t cnt = umin(hi - lo, L - cut - k);
    nl                 = below(cnt) << lo;
    const uint32_t j   = (0u - k) & 127u;
    if (j < cnt)
    {
        rs   = 1u << (lo + j);
        clen = umin(128u, L - k - j);
    }
}

// bm: run boundaries at the thread's nt positions (bit 0 always set at tile position 0); base =
// the thread's first tile position, n = tile length; Sprev = the last boundary before the thread,
// Enext = the first after it (n if none); left / right = run extension into the tile from before /
// after it (TileLink).
BRA_RT_HD RunCls cls_thread(uint32_t bm, uint32_t nt, uint32_t base, uint32_t n, uint32_t Sprev, uint32_t Enext, uint32_t left, uint32_t right)
{
    RunCls C{0, 0, 0, 0, 0, 0};
    if (!nt)
        return C;
    const uint32_t inner = bm & ~1u;               // boundaries after the thread's first position
    const uint32_t e1    = inner ? lo_bit(inner) : nt;  // end of the first segment
    {
        const uint32_t S = (bm & 1u) ? base : Sprev, E = inner ? base + e1 : Enext;
        const uint32_t lx = S == 0 ? left : 0u, rx = E == n ? right : 0u;
        seg_cls(0, e1, base - S + lx, E - S + lx + rx, C.nl, C.rs, C.c0);
        C.r0 = C.rs;
    }
    if (!inner)
        return C;
    const uint32_t bl = hi_bit(inner);  // start of the last segment
    {
        uint32_t nl1, rs1;
        seg_cls(bl, nt, 0u, Enext - (base + bl) + (Enext == n ? right : 0u), nl1, rs1, C.c1);
        C.nl |= nl1;
        C.rs |= rs1;
        C.r1 = rs1;
    }
    // inner runs, in [e1, bl): whole and shorter than 16 -- covered iff 3 or more long, one block
    // from the run's first position.  c: the position continues the previous one's run; g: the
    // third and later positions of a run, plus the two before each.
    const uint32_t M = below(bl) & ~below(e1);
    const uint32_t c = ~bm & M;
    uint32_t       g = c & (c << 1);
    g |= (g >> 1) | (g >> 2);
    C.nl |= g;
    C.rs |= g & bm;
    return C;
}

// Block length at run-block start i.
BRA_RT_HD uint32_t run_clen(const RunCls& C, uint32_t bm, uint32_t i)
{
    const uint32_t b = 1u << i;
    if (b == C.r0)
        return C.c0;
    if (b == C.r1)
        return C.c1;
    return lo_bit(bm & ~below(i + 1)) - i;  // inner run: up to the next boundary
}

// Literal-block control bytes of the thread's positions.  A gap starting inside the thread starts
// at gap offset 0; the thread's first gap may continue one from before it (GSprev: start of the
// gap holding the thread's first position if no covered position precedes it in the thread;
// g_in: gap offset at tile position 0).
BRA_RT_HD uint32_t ctl_mask(uint32_t lit, uint32_t nl, uint32_t nt, uint32_t base, uint32_t GSprev, uint32_t g_in)
{
    uint32_t ctl = lit & ~(lit << 1) & ~1u;
    if (lit & 1u)
    {
        const uint32_t go0 = base - GSprev + (GSprev == 0 ? g_in : 0u);
        const uint32_t ge  = nl ? lo_bit(nl) : nt;
        const uint32_t j   = (0u - go0) & 127u;
        if (j < ge)
            ctl |= 1u << j;
    }
    return ctl;
}

// Output bytes of the thread's positions: run-block start 2, covered 0, literal 1, control byte +1.
BRA_RT_HD uint32_t out_bytes(const RunCls& C, uint32_t nt, uint32_t base, uint32_t GSprev, uint32_t g_in)
{
    const uint32_t lit = below(nt) & ~C.nl;
    return 2 * popc(C.rs) + popc(lit) + popc(ctl_mask(lit, C.nl, nt, base, GSprev, g_in));
}

// Stage the thread's output at stage[pos...]; returns its length.  GEnext: the first covered
// position after the thread (n if none); rem_after: literals following the tile in its trailing gap.
BRA_RT_HD uint32_t stage_out(const uint32_t (&w)[4], uint32_t bm, const RunCls& C, uint32_t nt, uint32_t base, uint32_t n, uint32_t GSprev,
                             uint32_t GEnext, uint32_t g_in, uint32_t rem_after, uint8_t* stage, uint32_t pos)
{
    const uint32_t lit = below(nt) & ~C.nl;
    const uint32_t ctl = ctl_mask(lit, C.nl, nt, base, GSprev, g_in);
    const uint32_t hdr = C.rs | ctl;  // positions whose byte follows a block header
    uint32_t       off = pos;
#pragma unroll
    for (int i = 0; i < PT; ++i)
    {
        const uint32_t b = 1u << i;
        if ((C.rs | lit) & b)
        {
            const uint32_t h = (hdr & b) ? 1u : 0u;
            stage[off + h]   = (uint8_t) byte_at(w, i);
            off += 1 + h;
        }
    }
    for (uint32_t m = C.rs; m; m &= m - 1)
    {
        const uint32_t i = lo_bit(m), bb = below(i);
        stage[pos + 2 * popc(C.rs & bb) + popc(lit & bb) + popc(ctl & bb)] = (uint8_t) (int8_t) (1 - (int) run_clen(C, bm, i));
    }
    for (uint32_t m = ctl; m; m &= m - 1)
    {
        const uint32_t i = lo_bit(m), bb = below(i);
        const uint32_t em  = C.nl & ~below(i + 1);
        const uint32_t GE  = em ? base + lo_bit(em) : GEnext;  // end of the gap
        const uint32_t rem = GE - (base + i) + (GE == n ? rem_after : 0u);
        stage[pos + 2 * popc(C.rs & bb) + popc(lit & bb) + popc(ctl & bb)] = (uint8_t) (umin(rem, 128u) - 1);
    }
    return off - pos;
}

}  // namespace rle_tile
}  // namespace bra
