/*
 * oracle/bra_oracle.c -- TEST INFRASTRUCTURE ONLY (never linked into the product library).
 *
 * A CPU restatement of br-archive's per-block encoder chain (BWT -> MTF -> PackBits RLE ->
 * canonical Huffman) and its inverse, written from the reference's observable behaviour, not
 * copied from it.  Each function cites the reference file:line it restates
 * (paths are relative to the reference checkout, Raffaello/br-archive @ 0.4.0).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code, and
 * only as the checker.  It is pinned against (a) the reference's own known-answer values from
 * test/test_bra_encoders.cpp and (b) golden vectors produced by the reference encoders compiled
 * from /root/reference (see oracle/Makefile, tests/golden/make_golden.py).
 *
 * The restatement deliberately uses the *parallel-friendly* formulations the HIP path uses, so
 * that checking it against the reference also pins those formulations:
 *   - BWT: cyclic prefix doubling, ranks = group start (== #rotations strictly smaller);
 *   - RLE: structural form (maximal runs split in 128-chunks, literal gaps chopped at 128);
 *   - Huffman: the sorted-list insertion rule restated as an array lower_bound rule.
 */
#include "bra_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* BWT  (restates src/encoders/bra_bwt.c:31-53 comparator, :73-108 encode, :133-168 decode)    */
/* ------------------------------------------------------------------------------------------ */

/*
 * The reference sorts all n cyclic rotations with qsort_r (glibc: stable merge sort) using a
 * byte-wise cyclic comparator (bra_bwt.c:41-50) over an index array initialised 0..n-1
 * (bra_bwt.c:87-88).  Equal rotations therefore keep ascending index order, so the primary index
 * (bra_bwt.c:102-103) is the number of rotations strictly smaller than rotation 0.  Equal
 * rotations have equal last bytes, so L does not depend on the tie order at all.
 *
 * Restatement: prefix doubling on cyclic ranks.  rank[i] = start of i's group in the order by the
 * first h bytes.  Sorting by (rank[i], rank[i+h]) doubles h.  Stop when all groups are singletons
 * or h >= n (then groups are exactly the classes of identical rotations).
 */
int orc_bwt_encode(const uint8_t* in, uint32_t n, uint32_t* primary_index, uint8_t* out, uint32_t* sa_out)
{
    if (in == NULL || n == 0 || primary_index == NULL || out == NULL)
        return 0;

    uint32_t* sa    = (uint32_t*) malloc((size_t) n * sizeof(uint32_t));
    uint32_t* rank  = (uint32_t*) malloc((size_t) n * sizeof(uint32_t));
    uint32_t* nrank = (uint32_t*) malloc((size_t) n * sizeof(uint32_t));
    uint32_t* tmp   = (uint32_t*) malloc((size_t) n * sizeof(uint32_t));
    uint32_t* ptr   = (uint32_t*) malloc((size_t) n * sizeof(uint32_t));
    if (!sa || !rank || !nrank || !tmp || !ptr)
    {
        free(sa), free(rank), free(nrank), free(tmp), free(ptr);
        return 0;
    }

    /* h = 1: counting sort by the first byte. */
    uint32_t cnt[257] = {0};
    for (uint32_t i = 0; i < n; ++i)
        cnt[in[i] + 1]++;
    for (int c = 0; c < 256; ++c)
        cnt[c + 1] += cnt[c];
    for (uint32_t i = 0; i < n; ++i)
        rank[i] = cnt[in[i]];
    for (uint32_t i = 0; i < n; ++i)
        sa[cnt[in[i]]++] = i;

    uint32_t groups = 0;
    for (uint32_t j = 0; j < n; ++j)
        if (j == 0 || in[sa[j]] != in[sa[j - 1]])
            ++groups;

    for (uint64_t h = 1; groups < n && h < n; h <<= 1)
    {
        /* SA is sorted by rank; shifting each entry back by h gives an order sorted by rank[i+h]. */
        for (uint32_t j = 0; j < n; ++j)
            tmp[j] = (uint32_t) (((uint64_t) sa[j] + n - h) % n);
        /* Stable bucket pass by rank[i]; group starts are the bucket starts. */
        for (uint32_t j = 0; j < n; ++j)
            ptr[j] = j;
        for (uint32_t j = 0; j < n; ++j)
        {
            const uint32_t i = tmp[j];
            sa[ptr[rank[i]]++] = i;
        }
        groups           = 0;
        uint32_t g       = 0;
        uint32_t prev_r1 = 0, prev_r2 = 0;
        for (uint32_t j = 0; j < n; ++j)
        {
            const uint32_t i  = sa[j];
            const uint32_t r1 = rank[i];
            const uint32_t r2 = rank[(uint32_t) (((uint64_t) i + h) % n)];
            if (j == 0 || r1 != prev_r1 || r2 != prev_r2)
            {
                g = j;
                ++groups;
            }
            nrank[i] = g;
            prev_r1  = r1;
            prev_r2  = r2;
        }
        uint32_t* t = rank;
        rank        = nrank;
        nrank       = t;
    }

    for (uint32_t j = 0; j < n; ++j)
        out[j] = in[(uint32_t) (((uint64_t) sa[j] + n - 1) % n)];
    *primary_index = rank[0];
    if (sa_out)
        memcpy(sa_out, sa, (size_t) n * sizeof(uint32_t));

    free(sa), free(rank), free(nrank), free(tmp), free(ptr);
    return 1;
}

/* Inverse BWT (restates bra_bwt.c:133-168): stable LF transform, then n steps from pi. */
int orc_bwt_decode(const uint8_t* in, uint32_t n, uint32_t primary_index, uint8_t* out)
{
    if (in == NULL || out == NULL || n == 0 || primary_index >= n)
        return 0;
    uint32_t* lf = (uint32_t*) malloc((size_t) n * sizeof(uint32_t));
    if (!lf)
        return 0;
    uint32_t start[256] = {0}, cnt[256] = {0};
    for (uint32_t i = 0; i < n; ++i)
        cnt[in[i]]++;
    for (int c = 1; c < 256; ++c)
        start[c] = start[c - 1] + cnt[c - 1];
    for (uint32_t i = 0; i < n; ++i)
        lf[start[in[i]]++] = i;
    uint32_t k = primary_index;
    for (uint32_t i = 0; i < n; ++i)
    {
        k      = lf[k];
        out[i] = in[k];
    }
    free(lf);
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* MTF  (restates src/encoders/bra_mtf.c:9-13 init, :16-32 encode step, :35-46 decode step)    */
/* ------------------------------------------------------------------------------------------ */

int orc_mtf_encode(const uint8_t* in, size_t n, uint8_t* out)
{
    if (in == NULL || out == NULL || n == 0)
        return 0;
    uint8_t order[256];
    for (int c = 0; c < 256; ++c)
        order[c] = (uint8_t) c;
    for (size_t i = 0; i < n; ++i)
    {
        const uint8_t* hit = (const uint8_t*) memchr(order, in[i], 256);
        const size_t   p   = (size_t) (hit - order);
        memmove(order + 1, order, p);
        order[0] = in[i];
        out[i]   = (uint8_t) p;
    }
    return 1;
}

int orc_mtf_decode(const uint8_t* in, size_t n, uint8_t* out)
{
    if (in == NULL || out == NULL || n == 0)
        return 0;
    uint8_t order[256];
    for (int c = 0; c < 256; ++c)
        order[c] = (uint8_t) c;
    for (size_t i = 0; i < n; ++i)
    {
        const size_t  p = in[i];
        const uint8_t c = order[p];
        memmove(order + 1, order, p);
        order[0] = c;
        out[i]   = c;
    }
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* RLE / PackBits  (restates src/encoders/bra_rle.c:9-18 run detect, :20-56 size, :60-120     */
/* encode, :122-160 decode size, :162-224 decode)                                              */
/* ------------------------------------------------------------------------------------------ */

/*
 * Structural form of the reference's greedy encoder: every maximal run of length L >= 3 becomes
 * floor(L/128) run blocks of 128 plus one run block of r = L mod 128 when r >= 3; when r is 1 or
 * 2 those r tail bytes open the following literal gap.  A literal gap (everything not covered by
 * run blocks) is chopped into blocks of at most 128 bytes from its first byte.
 * Run block: (int8)-(len-1), byte.  Literal block: len-1, bytes.
 */
static size_t orc_rle_emit_gap(const uint8_t* in, size_t gs, size_t ge, uint8_t* out)
{
    size_t w = 0;
    for (size_t b = gs; b < ge; b += 128)
    {
        const size_t len = (ge - b) < 128 ? (ge - b) : 128;
        if (out)
        {
            out[w] = (uint8_t) (len - 1);
            memcpy(out + w + 1, in + b, len);
        }
        w += 1 + len;
    }
    return w;
}

size_t orc_rle_encode(const uint8_t* in, size_t n, uint8_t* out)
{
    size_t w        = 0;
    size_t gap      = 0;
    int    gap_open = 0;
    for (size_t s = 0; s < n;)
    {
        size_t e = s + 1;
        while (e < n && in[e] == in[s])
            ++e;
        const size_t L = e - s;
        if (L >= 3)
        {
            if (gap_open)
                w += orc_rle_emit_gap(in, gap, s, out ? out + w : NULL);
            gap_open = 0;
            for (size_t k = 0; k + 128 <= L; k += 128)
            {
                if (out)
                    out[w] = (uint8_t) (int8_t) -127, out[w + 1] = in[s];
                w += 2;
            }
            const size_t r = L % 128;
            if (r >= 3)
            {
                if (out)
                    out[w] = (uint8_t) (int8_t) (-(int) (r - 1)), out[w + 1] = in[s];
                w += 2;
            }
            else if (r > 0)
            {
                gap      = e - r;
                gap_open = 1;
            }
        }
        else if (!gap_open)
        {
            gap      = s;
            gap_open = 1;
        }
        s = e;
    }
    if (gap_open)
        w += orc_rle_emit_gap(in, gap, n, out ? out + w : NULL);
    return w;
}

/* Decoded size; 0 on a truncated block (bra_rle.c:122-160).  Control -128 is a no-op. */
size_t orc_rle_decode_size(const uint8_t* in, size_t n)
{
    size_t s = 0;
    for (size_t i = 0; i < n;)
    {
        const int c = (int8_t) in[i++];
        if (c >= 0)
        {
            if (i + (size_t) c + 1 > n)
                return 0;
            s += (size_t) c + 1;
            i += (size_t) c + 1;
        }
        else if (c >= -127)
        {
            if (i >= n)
                return 0;
            s += (size_t) (1 - c);
            ++i;
        }
    }
    return s;
}

size_t orc_rle_decode(const uint8_t* in, size_t n, uint8_t* out)
{
    const size_t s = orc_rle_decode_size(in, n);
    if (s == 0)
        return 0;
    size_t w = 0;
    for (size_t i = 0; i < n;)
    {
        const int c = (int8_t) in[i++];
        if (c >= 0)
        {
            memcpy(out + w, in + i, (size_t) c + 1);
            w += (size_t) c + 1;
            i += (size_t) c + 1;
        }
        else if (c >= -127)
        {
            memset(out + w, in[i++], (size_t) (1 - c));
            w += (size_t) (1 - c);
        }
    }
    return s;
}

/* ------------------------------------------------------------------------------------------ */
/* Huffman  (restates src/encoders/bra_huffman.c)                                              */
/* ------------------------------------------------------------------------------------------ */

/*
 * Code lengths from the reference's frequency-sorted list (bra_huffman.c:90-186).
 * Insertion rule of bra_minHeap_insert (:102-117) restated on an array `list` of node ids:
 *   position = 0                        if the list is empty or list[0].freq > f
 *            = max(1, lower_bound(f))   otherwise
 * (an equal-frequency node goes in front of the first node with freq >= f, except that a head
 * with freq == f stays the head).  Leaves enter in symbol order (:140-153); each merge pops two
 * nodes, l then r, and inserts a node of freq l+r (:158-175); left edge = 0, right edge = 1
 * (:216-219); a single leaf gets length 1 (:201-207).
 * Returns 0 when no symbol is present (tree build fails, :155-156).
 */
int orc_huffman_lengths(const uint32_t freq[256], uint8_t lengths[256])
{
    uint32_t nf[512];
    int16_t  left[512], right[512], parent[512];
    int      list[512];
    int      len = 0, nodes = 0;

    memset(lengths, 0, 256);
    for (int s = 0; s < 256; ++s)
    {
        if (freq[s] == 0)
            continue;
        const int id = nodes++;
        nf[id] = freq[s], left[id] = right[id] = -1, parent[id] = -1;
        int p = 0;
        if (len > 0 && nf[list[0]] <= freq[s])
        {
            p = 1;
            while (p < len && nf[list[p]] < freq[s])
                ++p;
        }
        memmove(list + p + 1, list + p, (size_t) (len - p) * sizeof(int));
        list[p] = id;
        ++len;
    }
    if (len == 0)
        return 0;
    const int leaves = nodes;
    while (len > 1)
    {
        const int l = list[0], r = list[1];
        memmove(list, list + 2, (size_t) (len - 2) * sizeof(int));
        len -= 2;
        const int      id = nodes++;
        const uint32_t f  = nf[l] + nf[r];
        nf[id] = f, left[id] = (int16_t) l, right[id] = (int16_t) r, parent[id] = -1;
        parent[l] = parent[r] = (int16_t) id;
        int p = 0;
        if (len > 0 && nf[list[0]] <= f)
        {
            p = 1;
            while (p < len && nf[list[p]] < f)
                ++p;
        }
        memmove(list + p + 1, list + p, (size_t) (len - p) * sizeof(int));
        list[p] = id;
        ++len;
    }
    /* leaf ids 0..leaves-1 were assigned in ascending symbol order */
    int id = 0;
    for (int s = 0; s < 256; ++s)
    {
        if (freq[s] == 0)
            continue;
        unsigned depth = 0;
        for (int v = id; parent[v] >= 0; v = parent[v])
            ++depth;
        lengths[s] = (uint8_t) (depth == 0 ? 1 : depth);
        ++id;
    }
    (void) left, (void) right, (void) leaves;
    return 1;
}

/*
 * Canonical codes (bra_huffman.c:227-261): next code per length computed in uint32_t (wraps),
 * codes assigned in ascending symbol order.  A code of length len is emitted MSB-first as the
 * len-bit number `code` (bits above 31 are therefore zero).
 */
void orc_huffman_codes(const uint8_t lengths[256], uint32_t codes[256])
{
    uint32_t count[257] = {0}, next[257] = {0};
    for (int s = 0; s < 256; ++s)
        if (lengths[s])
            count[lengths[s]]++;
    uint32_t code = 0;
    for (int l = 1; l <= 256; ++l)
    {
        code <<= 1;
        next[l] = code;
        code += (l <= 256) ? count[l] : 0;
    }
    for (int s = 0; s < 256; ++s)
        codes[s] = lengths[s] ? next[lengths[s]]++ : 0;
}

/* Encode (bra_huffman.c:352-432).  Returns 0 on failure (buf_size == 0). */
int orc_huffman_encode(const uint8_t* in, uint32_t n, orc_huffman_meta_t* meta, uint8_t** payload)
{
    uint32_t freq[256] = {0};
    for (uint32_t i = 0; i < n; ++i)
        freq[in[i]]++;
    if (!orc_huffman_lengths(freq, meta->lengths))
        return 0;
    uint32_t codes[256];
    orc_huffman_codes(meta->lengths, codes);
    uint32_t bits = 0;
    for (uint32_t i = 0; i < n; ++i)
        bits += meta->lengths[in[i]];
    meta->orig_size    = n;
    meta->encoded_size = (bits + 7u) / 8u; /* u32 arithmetic, as bra_huffman.c:395 */
    uint8_t* out       = (uint8_t*) calloc(meta->encoded_size ? meta->encoded_size : 1, 1);
    if (!out)
        return 0;
    uint64_t bitpos = 0;
    for (uint32_t i = 0; i < n; ++i)
    {
        const unsigned l = meta->lengths[in[i]];
        const uint32_t c = codes[in[i]];
        for (unsigned j = 0; j < l; ++j)
        {
            const unsigned b = l - 1 - j; /* bit index within the len-bit number */
            if (b < 32 && ((c >> b) & 1u))
                out[bitpos >> 3] |= (uint8_t) (0x80u >> (bitpos & 7));
            ++bitpos;
        }
    }
    *payload = out;
    return 1;
}

/*
 * Decode (bra_huffman.c:263-348 tree from lengths, :434-498 walk).  The reference inserts each
 * symbol's canonical code into a binary tree, failing when the final edge is already taken
 * (:292-305); an existing node on the path is reused whatever it is (so a leaf may acquire
 * children and stop being a leaf).  The walk emits a symbol at every childless node and stops at
 * orig_size.  A NULL edge or a final count != orig_size is an error.  Where the reference would
 * write past orig_size (a stream longer than its symbols need) this restatement reports an error.
 * Returns 1 and fills out[0..orig_size) on success.
 */
int orc_huffman_decode(const orc_huffman_meta_t* meta, const uint8_t* data, uint8_t* out)
{
    enum { MAXN = 256 * 256 + 2 };
    int32_t* child = (int32_t*) malloc(sizeof(int32_t) * 2 * MAXN);
    uint8_t* sym   = (uint8_t*) malloc(MAXN);
    if (!child || !sym)
    {
        free(child), free(sym);
        return 0;
    }
    int nodes = 1;
    child[0] = child[1] = -1;
    sym[0]              = 0;
    uint32_t codes[256];
    orc_huffman_codes(meta->lengths, codes);
    int ok = 1;
    for (int s = 0; s < 256 && ok; ++s)
    {
        const unsigned l = meta->lengths[s];
        if (!l)
            continue;
        int cur = 0;
        for (unsigned j = 0; j < l; ++j)
        {
            const unsigned b   = l - 1 - j;
            const int      bit = (b < 32) ? (int) ((codes[s] >> b) & 1u) : 0;
            if (j == l - 1)
            {
                if (child[2 * cur + bit] != -1)
                {
                    ok = 0;
                    break;
                }
                child[2 * cur + bit] = nodes;
                child[2 * nodes] = child[2 * nodes + 1] = -1;
                sym[nodes++]                            = (uint8_t) s;
            }
            else
            {
                if (child[2 * cur + bit] == -1)
                {
                    child[2 * cur + bit] = nodes;
                    child[2 * nodes] = child[2 * nodes + 1] = -1;
                    sym[nodes++]                            = 0;
                }
                cur = child[2 * cur + bit];
            }
        }
    }
    uint32_t k = 0;
    if (ok)
    {
        int cur = 0;
        for (uint32_t i = 0; i < meta->encoded_size && ok; ++i)
        {
            for (int bit = 7; bit >= 0; --bit)
            {
                cur = child[2 * cur + ((data[i] >> bit) & 1)];
                if (cur == -1)
                {
                    ok = 0;
                    break;
                }
                if (child[2 * cur] == -1 && child[2 * cur + 1] == -1)
                {
                    if (k >= meta->orig_size)
                    {
                        ok = 0; /* reference would overrun its buffer here */
                        break;
                    }
                    out[k++] = sym[cur];
                    cur      = 0;
                    if (k >= meta->orig_size)
                        break;
                }
            }
        }
    }
    free(child), free(sym);
    return ok && k == meta->orig_size;
}

/* ------------------------------------------------------------------------------------------ */
/* Whole chunk, as bra_io_file_chunks_compress_file does it (lib_bra_io_file_chunks.c:217-245) */
/* ------------------------------------------------------------------------------------------ */

int orc_encode_block(const uint8_t* in, uint32_t n, uint32_t* primary_index, orc_huffman_meta_t* meta, uint8_t** payload,
                     uint8_t* bwt_out, uint8_t* mtf_out, uint8_t** rle_out, size_t* rle_size)
{
    uint8_t* b = bwt_out ? bwt_out : (uint8_t*) malloc(n);
    uint8_t* m = mtf_out ? mtf_out : (uint8_t*) malloc(n);
    uint8_t* r = (uint8_t*) malloc((size_t) n + n / 128 + 2);
    int      ok = b && m && r && orc_bwt_encode(in, n, primary_index, b, NULL) && orc_mtf_encode(b, n, m);
    size_t   rs = ok ? orc_rle_encode(m, n, r) : 0;
    ok          = ok && rs > 0 && orc_huffman_encode(r, (uint32_t) rs, meta, payload);
    if (!bwt_out)
        free(b);
    if (!mtf_out)
        free(m);
    if (ok && rle_out)
    {
        *rle_out  = r;
        *rle_size = rs;
    }
    else
        free(r);
    return ok;
}

/* ------------------------------------------------------------------------------------------ */
/* CRC32C and the chunk stream  (restates src/utils/lib_bra_crc32c.c:102-231 and the CRC        */
/* sequence of src/io/lib_bra_io_file_chunks.c:214,248-249,291-292)                             */
/* ------------------------------------------------------------------------------------------ */

/* Reflected Castagnoli polynomial (lib_bra_crc32c.c:27). */
#define ORC_CRC_POLY 0x82F63B78u

static uint32_t orc_crc_tab[256];
static int      orc_crc_ready;

static void orc_crc_init(void)
{
    if (orc_crc_ready)
        return;
    for (uint32_t v = 0; v < 256; ++v)
    {
        uint32_t c = v;
        for (int k = 0; k < 8; ++k)
            c = (c & 1) ? (c >> 1) ^ ORC_CRC_POLY : c >> 1;
        orc_crc_tab[v] = c;
    }
    orc_crc_ready = 1;
}

/* bra_crc32c(data, length, previous_crc) (lib_bra_crc32c.c:102-117): the public value is the
 * complemented register, so chaining passes the previous result straight back in. */
uint32_t orc_crc32c(const void* data, uint64_t length, uint32_t previous_crc)
{
    orc_crc_init();
    const uint8_t* p = (const uint8_t*) data;
    uint32_t       c = ~previous_crc;
    for (uint64_t i = 0; i < length; ++i)
        c = orc_crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

/* GF(2) 32x32 operator helpers: column n of `mat` is the image of bit n. */
static uint32_t orc_gf2_times(const uint32_t* mat, uint32_t vec)
{
    uint32_t sum = 0;
    for (int n = 0; vec; ++n, vec >>= 1)
        if (vec & 1)
            sum ^= mat[n];
    return sum;
}

static void orc_gf2_square(uint32_t* sq, const uint32_t* mat)
{
    for (int n = 0; n < 32; ++n)
        sq[n] = orc_gf2_times(mat, mat[n]);
}

/* bra_crc32c_combine(a, b, len_b) (lib_bra_crc32c.c:181-231): the CRC of A||B from crc(A),
 * crc(B) and |B|.  Appending |B| zero bytes to A is applied as repeated squarings of the
 * one-zero-bit operator (1 -> 2 -> 4 -> 8 bits, then one squaring per bit of len_b). */
uint32_t orc_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint32_t len_b)
{
    if (len_b == 0)
        return crc_a;
    uint32_t op1[32], op2[32];
    op1[0] = ORC_CRC_POLY; /* one zero bit */
    for (int n = 1; n < 32; ++n)
        op1[n] = 1u << (n - 1);
    orc_gf2_square(op2, op1); /* two zero bits  */
    orc_gf2_square(op1, op2); /* four zero bits */
    uint32_t* cur = op1;
    uint32_t* nxt = op2;
    while (len_b)
    {
        orc_gf2_square(nxt, cur); /* 8, 16, 32 ... zero bits */
        if (len_b & 1)
            crc_a = orc_gf2_times(nxt, crc_a);
        len_b >>= 1;
        uint32_t* t = cur;
        cur         = nxt;
        nxt         = t;
    }
    return crc_a ^ crc_b;
}

/* The `crc32` variable of bra_io_file_chunks_compress_file after its loop (:186,214,248-249):
 * per chunk the 268-byte in-memory header, then the source chunk, folded in by combine.
 * headers: nchunks x 268 bytes; data: the source (or, on decode, the decoded) chunks back to back
 * with every chunk chunk_size bytes except a ragged last one. */
uint32_t orc_chunks_crc32c(const uint8_t* headers, const uint8_t* data, uint64_t total, uint32_t chunk_size, uint32_t crc)
{
    uint64_t b = 0;
    for (uint64_t i = 0; i < total; i += chunk_size, ++b)
    {
        const uint32_t s   = (uint32_t) ((total - i) < chunk_size ? (total - i) : chunk_size);
        const uint32_t src = orc_crc32c(data + i, s, 0);
        crc                = orc_crc32c(headers + 268 * b, 268, crc);
        crc                = orc_crc32c_combine(crc, src, s);
    }
    return crc;
}

/* The meta entry CRC after a compressed file (:291-292): the 8-byte tmpfile size, then the chunk
 * stream CRC combined over data_size + num_chunks * 268 bytes (len_b is uint32_t there). */
uint32_t orc_entry_crc32c(uint32_t me_crc, int64_t tmpfile_size, uint32_t chunks_crc, uint64_t data_size)
{
    uint64_t num_chunks = data_size / (256 * 1024) + (data_size % (256 * 1024) ? 1 : 0);
    me_crc              = orc_crc32c(&tmpfile_size, sizeof tmpfile_size, me_crc);
    return orc_crc32c_combine(me_crc, chunks_crc, (uint32_t) (data_size + num_chunks * 268));
}

/* One .BRa chunk record (lib_bra_io_file_chunks.c:76-95 + :260): 3 low bytes of the primary
 * index, the packed 264-byte bra_huffman_t, the payload.  Returns the record size. */
size_t orc_frame_record(const uint8_t header268[268], const uint8_t* payload, uint32_t encoded_size, uint8_t* out)
{
    memcpy(out, header268, 3);
    memcpy(out + 3, header268 + 4, 264);
    if (encoded_size)
        memcpy(out + 267, payload, encoded_size);
    return 267 + (size_t) encoded_size;
}

void orc_free(void* p) { free(p); }
