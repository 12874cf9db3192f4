/*
 * bra_synth.c -- deterministic synthetic inputs for the benchmark and the parity tests
 * (SURVEY.md section 8.1 row d).  Not part of the encoder path.
 *
 * Generator: xorshift64* (s ^= s >> 12; s ^= s << 25; s ^= s >> 27; return s * 0x2545F4914F6CDD1D),
 * per-block seed = 0x9E3779B97F4A7C15 ^ (block_index * 0xD1B54A32D192ED03).
 *
 * kinds:
 *   BRA_SYNTH_TEXT    "enwik-style" text: Zipf(s = 1.1) word stream over the 155-word vocabulary of
 *                     the reference's test/fixtures/lorem.txt (ranked by frequency there), ' '
 *                     separators, '\n' after ~1/12 of the words, '.' / ',' after ~1/16 of them;
 *   BRA_SYNTH_RANDOM  uniform bytes (top byte of each xorshift64* draw);
 *   BRA_SYNTH_SYM16   16-symbol geometric alphabet 'a' + min(ctz(r), 15) (H ~ 2 bit/byte);
 *   BRA_SYNTH_TILED   the 19-byte reference fixture test/test.txt ("Test File Fixture.\n") tiled.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

enum { BRA_SYNTH_TEXT = 0, BRA_SYNTH_RANDOM = 1, BRA_SYNTH_SYM16 = 2, BRA_SYNTH_TILED = 3 };

static const char* const k_vocab[] = {
    "et", "ut", "ac", "id", "ipsum", "non", "tincidunt", "amet", "arcu", "eget", "in", "nec", "nunc",
    "pulvinar", "sed", "sem", "sit", "vel", "auctor", "dolor", "elit", "erat", "lorem", "metus", "nibh",
    "odio", "pellentesque", "quis", "urna", "velit", "ante", "consectetur", "donec", "etiam", "eu", "felis",
    "fringilla", "gravida", "imperdiet", "laoreet", "mattis", "morbi", "nulla", "orci", "quam", "sodales",
    "tellus", "venenatis", "vestibulum", "vitae", "aliquam", "at", "condimentum", "consequat", "euismod",
    "faucibus", "fusce", "lacinia", "lectus", "libero", "ligula", "luctus", "maecenas", "malesuada",
    "mauris", "molestie", "praesent", "quisque", "risus", "rutrum", "sagittis", "tristique", "a", "accumsan",
    "adipiscing", "augue", "convallis", "curabitur", "cursus", "dapibus", "diam", "dignissim", "dui", "duis",
    "efficitur", "egestas", "ex", "fames", "fermentum", "feugiat", "hendrerit", "lacus", "magna", "massa",
    "ornare", "per", "placerat", "porta", "sapien", "scelerisque", "semper", "tempor", "ullamcorper",
    "ultricies", "vehicula", "vivamus", "ad", "aenean", "aliquet", "aptent", "bibendum", "class", "congue",
    "conubia", "dictum", "dictumst", "eleifend", "enim", "eros", "facilisis", "habitant", "habitasse", "hac",
    "himenaeos", "inceptos", "integer", "interdum", "justo", "leo", "litora", "mi", "mollis", "nam", "netus",
    "nisi", "nostra", "nullam", "pharetra", "phasellus", "platea", "porttitor", "posuere", "pretium",
    "primis", "rhoncus", "senectus", "sociosqu", "suspendisse", "taciti", "torquent", "tortor", "turpis",
    "varius", "viverra", "volutpat",
};
#define K_NWORDS ((int) (sizeof(k_vocab) / sizeof(k_vocab[0])))

static inline uint64_t xs_next(uint64_t* s)
{
    uint64_t x = *s;
    x ^= x >> 12;
    x ^= x << 25;
    x ^= x >> 27;
    *s = x;
    return x * 0x2545F4914F6CDD1DULL;
}

static double   g_cdf[256];
static int      g_cdf_ready = 0;
static unsigned g_wlen[256];

static void init_cdf(void)
{
    double acc = 0.0;
    for (int k = 0; k < K_NWORDS; ++k)
    {
        acc += pow((double) (k + 1), -1.1);
        g_cdf[k]  = acc;
        g_wlen[k] = (unsigned) strlen(k_vocab[k]);
    }
    for (int k = 0; k < K_NWORDS; ++k)
        g_cdf[k] /= acc;
    g_cdf[K_NWORDS - 1] = 1.0;
    g_cdf_ready         = 1;
}

uint64_t bra_synth_seed(uint64_t block_index)
{
    uint64_t s = 0x9E3779B97F4A7C15ULL ^ (block_index * 0xD1B54A32D192ED03ULL);
    return s ? s : 1;
}

int bra_synth_block(int kind, uint64_t block_index, uint8_t* out, uint64_t n)
{
    uint64_t s = bra_synth_seed(block_index);
    switch (kind)
    {
    case BRA_SYNTH_RANDOM:
        for (uint64_t i = 0; i < n; ++i)
            out[i] = (uint8_t) (xs_next(&s) >> 56);
        return 1;
    case BRA_SYNTH_SYM16:
        for (uint64_t i = 0; i < n; ++i)
        {
            const uint64_t r = xs_next(&s);
            const int      z = r ? __builtin_ctzll(r) : 64;
            out[i]           = (uint8_t) ('a' + (z < 15 ? z : 15));
        }
        return 1;
    case BRA_SYNTH_TILED:
    {
        static const char t[] = "Test File Fixture.\n";
        for (uint64_t i = 0; i < n; ++i)
            out[i] = (uint8_t) t[i % 19];
        return 1;
    }
    case BRA_SYNTH_TEXT:
    {
        if (!g_cdf_ready)
            init_cdf();
        uint64_t pos = 0;
        while (pos < n)
        {
            const uint64_t r = xs_next(&s);
            const double   u = (double) (r >> 11) * (1.0 / 9007199254740992.0);
            int lo = 0, hi = K_NWORDS - 1;
            while (lo < hi)
            {
                const int mid = (lo + hi) / 2;
                if (g_cdf[mid] < u)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            const char* w = k_vocab[lo];
            for (unsigned k = 0; k < g_wlen[lo] && pos < n; ++k)
                out[pos++] = (uint8_t) w[k];
            const uint64_t r2 = xs_next(&s);
            if ((r2 & 15u) == 0 && pos < n)
                out[pos++] = (uint8_t) (((r2 >> 4) & 1u) ? '.' : ',');
            if (pos < n)
                out[pos++] = (uint8_t) (((r2 >> 8) % 12u) == 0 ? '\n' : ' ');
        }
        return 1;
    }
    default:
        return 0;
    }
}

/* Fill `nblocks` consecutive blocks of `block_size` bytes (the last one `total - ...` bytes). */
int bra_synth_fill(int kind, uint64_t first_block, uint8_t* out, uint64_t total, uint64_t block_size)
{
    uint64_t b = first_block;
    for (uint64_t off = 0; off < total; off += block_size, ++b)
    {
        const uint64_t len = (total - off) < block_size ? (total - off) : block_size;
        if (!bra_synth_block(kind, b, out + off, len))
            return 0;
    }
    return 1;
}

/* Fill `total` bytes with the blocks first_block, first_block + stride, ... (a round-robin shard of a
 * global stream: rank r of G ranks holds global blocks r, r + G, ...), back to back. */
int bra_synth_fill_strided(int kind, uint64_t first_block, uint64_t stride, uint8_t* out, uint64_t total, uint64_t block_size)
{
    uint64_t b = first_block;
    for (uint64_t off = 0; off < total; off += block_size, b += stride)
    {
        const uint64_t len = (total - off) < block_size ? (total - off) : block_size;
        if (!bra_synth_block(kind, b, out + off, len))
            return 0;
    }
    return 1;
}
