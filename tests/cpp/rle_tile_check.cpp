// CPU check of the RLE tile classification (br-archive_amd/csrc/rle_tile.h): whole blocks are
// encoded tile by tile the way rle.hip's kernels do it (thread scans, per-thread classification,
// staged output) with the cross-tile state computed directly from the block, and compared byte
// for byte with the oracle encoder (oracle/bra_oracle.c, orc_rle_encode).  Test infrastructure
// only (tests/test_rle_tile.py builds and runs it).
//
//   rle_tile_check [iterations] [seed]   -> "ok <blocks> <bytes>" or a first mismatch, exit 1
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../br-archive_amd/csrc/rle_tile.h"
extern "C" {
#include "../../oracle/bra_oracle.h"
}

using namespace bra::rle_tile;

static constexpr uint32_t TILE = 4096, TPB = TILE / PT;

static uint64_t rng_state = 1;
static uint32_t rnd()
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t) rng_state;
}

// Blocks mixing literal stretches and runs of every interesting length (1..3, around 128 and its
// multiples, beyond a tile) over a small or a full alphabet.
static std::vector<uint8_t> make_block(uint32_t n)
{
    std::vector<uint8_t> b(n);
    const uint32_t       alpha = (rnd() & 1) ? 4 : 256;
    const uint32_t       style = rnd() % 6;
    for (uint32_t i = 0; i < n;)
    {
        uint32_t len, noise = 0;  // a run of len, or noise (literals) of that length
        switch (style == 3 ? rnd() % 3 : style)
        {
        case 0: len = 1 + rnd() % 4; break;
        case 1: len = (rnd() & 1) ? 1 + rnd() % 300 : 126 + rnd() % 6; break;
        case 2: len = (rnd() % 8 == 0) ? 1 + rnd() % 9000 : 1 + rnd() % 3; break;
        case 4: len = n, noise = 1; break;
        default:
            noise = rnd() & 1;
            len   = noise ? 1 + rnd() % 600 : (rnd() & 1) ? 1 + rnd() % 6 : 1 + rnd() % 400;
            break;
        }
        const uint8_t v = (uint8_t) (rnd() % alpha);
        for (uint32_t j = 0; j < len && i < n; ++j, ++i)
        {
            b[i] = noise ? (uint8_t) rnd() : v;
            if (noise && i > 0 && b[i] == b[i - 1])
                b[i] ^= 0x55;  // keep noise run-free
        }
    }
    return b;
}

// The tile-by-tile encode of rle.hip restated on the host.
static std::vector<uint8_t> encode_tiled(const std::vector<uint8_t>& in)
{
    const uint32_t        n = (uint32_t) in.size();
    std::vector<uint8_t>  out;
    // block-level facts the link / offsets kernels derive: covered positions (maximal runs)
    std::vector<uint8_t>  cov(n, 0);
    for (uint32_t s = 0; s < n;)
    {
        uint32_t e = s + 1;
        while (e < n && in[e] == in[s])
            ++e;
        const uint32_t L = e - s, tail = L % 128, cut = tail < 3 ? tail : 0;
        if (L >= 3)
            for (uint32_t k = 0; k < L - cut; ++k)
                cov[s + k] = 1;
        s = e;
    }
    std::vector<uint8_t> stage(TILE * 2 + 64);
    for (uint32_t t0 = 0; t0 < n; t0 += TILE)
    {
        const uint32_t tn = std::min(TILE, n - t0);
        const uint8_t* p  = in.data() + t0;
        uint32_t       left = 0, right = 0, g_in = 0, rem_after = 0;
        while (left < t0 && in[t0 - 1 - left] == p[0])
            ++left;
        while (t0 + tn + right < n && in[t0 + tn + right] == p[tn - 1])
            ++right;
        while (g_in < t0 && !cov[t0 - 1 - g_in])
            ++g_in;
        while (t0 + tn + rem_after < n && !cov[t0 + tn + rem_after])
            ++rem_after;
        uint32_t w[TPB][4], bm[TPB], nt[TPB], base[TPB];
        for (uint32_t t = 0; t < TPB; ++t)
        {
            base[t] = t * PT;
            nt[t]   = base[t] < tn ? std::min<uint32_t>(PT, tn - base[t]) : 0;
            for (int d = 0; d < 4; ++d)
            {
                uint32_t x = 0;
                for (int j = 0; j < 4; ++j)
                    if (base[t] + 4 * d + j < tn)
                        x |= (uint32_t) p[base[t] + 4 * d + j] << (8 * j);
                w[t][d] = x;
            }
            const uint32_t prev = base[t] > 0 && nt[t] ? p[base[t] - 1] : 0u;
            uint32_t       m    = diff_mask(w[t], prev);
            if (base[t] == 0)
                m |= 1u;
            bm[t] = nt[t] ? m & below(nt[t]) : 0u;
        }
        RunCls C[TPB];
        {
            uint32_t Sprev[TPB], Enext[TPB], run = 0;
            for (uint32_t t = 0; t < TPB; ++t)
            {
                Sprev[t] = run;
                run      = std::max(run, bm[t] ? base[t] + hi_bit(bm[t]) : 0u);
            }
            run = tn;
            for (int t = TPB - 1; t >= 0; --t)
            {
                Enext[t] = run;
                run      = std::min(run, bm[t] ? base[t] + lo_bit(bm[t]) : tn);
            }
            for (uint32_t t = 0; t < TPB; ++t)
                C[t] = cls_thread(bm[t], nt[t], base[t], tn, Sprev[t], Enext[t], left, right);
        }
        uint32_t GSprev[TPB], GEnext[TPB];
        {
            uint32_t run = 0;
            for (uint32_t t = 0; t < TPB; ++t)
            {
                GSprev[t] = run;
                run       = std::max(run, C[t].nl ? base[t] + hi_bit(C[t].nl) + 1 : 0u);
            }
            run = tn;
            for (int t = TPB - 1; t >= 0; --t)
            {
                GEnext[t] = run;
                run       = std::min(run, C[t].nl ? base[t] + lo_bit(C[t].nl) : tn);
            }
        }
        uint32_t pos = 0;
        for (uint32_t t = 0; t < TPB; ++t)
        {
            const uint32_t by = out_bytes(C[t], nt[t], base[t], GSprev[t], g_in);
            const uint32_t wr = stage_out(w[t], bm[t], C[t], nt[t], base[t], tn, GSprev[t], GEnext[t], g_in, rem_after, stage.data(), pos);
            if (wr != by)
            {
                fprintf(stderr, "tile %u thread %u: out_bytes %u, staged %u\n", t0 / TILE, t, by, wr);
                exit(1);
            }
            pos += by;
        }
        out.insert(out.end(), stage.begin(), stage.begin() + pos);
    }
    return out;
}

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 300;
    rng_state       = argc > 2 ? strtoull(argv[2], nullptr, 0) : 0x9E3779B97F4A7C15ull;
    uint64_t bytes  = 0;
    for (int it = 0; it < iters; ++it)
    {
        const uint32_t n = (it % 7 == 0) ? 1 + rnd() % 64 : (it % 3 == 0) ? TILE * (1 + rnd() % 3) : 1 + rnd() % (TILE * 4);
        const std::vector<uint8_t> in = make_block(n);
        std::vector<uint8_t>       ref(n + n / 128 + 16);
        ref.resize(orc_rle_encode(in.data(), n, ref.data()));
        const std::vector<uint8_t> got = encode_tiled(in);
        if (got != ref)
        {
            size_t i = 0;
            while (i < got.size() && i < ref.size() && got[i] == ref[i])
                ++i;
            fprintf(stderr, "block %d (n %u): sizes %zu / %zu, first difference at %zu\n", it, n, got.size(), ref.size(), i);
            return 1;
        }
        bytes += n;
    }
    printf("ok %d %llu\n", iters, (unsigned long long) bytes);
    return 0;
}
