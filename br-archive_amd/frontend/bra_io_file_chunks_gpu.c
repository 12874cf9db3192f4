/*
 * bra_io_file_chunks_gpu.c -- the batched chunk loop of lib_bra on the MI355X block codec
 * (SURVEY 8.1 row f1).  A drop-in replacement for the reference's src/io/lib_bra_io_file_chunks.c:
 * it defines the six functions of src/io/lib_bra_io_file_chunks.h with the same signatures, file
 * formats, CRC sequence and error behaviour, and is compiled against lib_bra's own headers (the
 * maintainer's tree; oracle/Makefile target `gpulib` builds it against /root/reference/src).
 *
 * Where the reference encodes one 256 KiB chunk at a time through the four encoders
 * (lib_bra_io_file_chunks.c:199-266), this file reads BATCH_CHUNKS chunks, makes ONE call into
 * libbra_hip.so (bra_gpu_compress_chunks_host: all chunks encoded, framed and CRC'd on the GPU)
 * and writes the returned chunk records to the temporary file.  The STORED fallback (:268-278),
 * the meta entry update (:280-297) and the copy into the archive are the reference's sequence.
 * Decoding parses the records of a batch on the host, hands them to bra_gpu_decompress_chunks_host
 * and folds me->crc32 the way the reference does per chunk (:396-397).  When a batch holds a bad
 * record, its records are decoded again one at a time through the per-chunk entry points of
 * libbra_hip.so, so dst receives the same prefix of good chunks and the log the same message as
 * the reference's loop.  There is no CPU encoder here: without a GPU the calls fail and log, like
 * every other entry point of libbra_hip.so.
 */
#include <lib_bra_defs.h>
#include <lib_bra_private.h>
#include <lib_bra_types.h>

#include <io/lib_bra_io_file.h>
#include <io/lib_bra_io_file_chunks.h>
#include <io/lib_bra_io_file_meta_entries.h>
#include <log/bra_log.h>
#include <utils/lib_bra_crc32c.h>

#include <encoders/bra_huffman.h>
#include <encoders/bra_rle.h>

#define BRA_HIP_NO_TYPES /* the ABI types come from lib_bra_types.h / bra_huffman.h above */
#include "../../include/bra_hip.h"

#include <assert.h>
#include <inttypes.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define CHUNK_SIZE ((uint64_t) BRA_MAX_CHUNK_SIZE)
#ifndef BATCH_CHUNKS
#define BATCH_CHUNKS 256u /* 64 MiB of input per device call (tests build a 2-chunk variant) */
#endif

/* One device context for the front end, created once (pthread_once) on the device current when
 * lib_bra first compresses or decompresses, and destroyed at process exit. */
static bra_gpu_ctx_t*  g_front_ctx  = NULL;
static pthread_once_t  g_front_once = PTHREAD_ONCE_INIT;

static void front_ctx_destroy(void)
{
    bra_gpu_ctx_destroy(g_front_ctx);
    g_front_ctx = NULL;
}

static void front_ctx_create(void)
{
    g_front_ctx = bra_gpu_ctx_create(-1);
    if (g_front_ctx != NULL)
        atexit(front_ctx_destroy);
}

static bra_gpu_ctx_t* front_ctx(void)
{
    pthread_once(&g_front_once, front_ctx_create);
    if (g_front_ctx == NULL)
        bra_log_critical("no GPU context for the chunk loop (libbra_hip.so)");
    return g_front_ctx;
}

/* ---- chunk headers: 3-byte little-endian pi, then the packed bra_huffman_t (:59-95) ---- */
bool bra_io_file_chunks_read_header(bra_io_file_t* src, bra_io_chunk_header_t* chunk_header)
{
    assert(src != NULL && chunk_header != NULL);
    uint8_t pi[BRA_BWT_INDEX_BYTES];
    if (!bra_io_file_read(src, pi, sizeof pi))
    {
        bra_log_error("unable to read chunk primary index from %s", src->fn);
        return false;
    }
    chunk_header->primary_index = (bra_bwt_index_t) pi[0] | (bra_bwt_index_t) pi[1] << 8 | (bra_bwt_index_t) pi[2] << 16;
    if (!bra_io_file_read(src, &chunk_header->huffman, sizeof(bra_huffman_t)))
    {
        bra_log_error("unable to read chunk huffman header from %s", src->fn);
        return false;
    }
    return true;
}

bool bra_io_file_chunks_write_header(bra_io_file_t* dst, const bra_io_chunk_header_t* chunk_header)
{
    assert(dst != NULL && chunk_header != NULL);
    const uint8_t pi[BRA_BWT_INDEX_BYTES] = {(uint8_t) chunk_header->primary_index, (uint8_t) (chunk_header->primary_index >> 8),
                                             (uint8_t) (chunk_header->primary_index >> 16)};
    if (!bra_io_file_write(dst, pi, sizeof pi))
    {
        bra_log_error("unable to write chunk primary index to %s", dst->fn);
        return false;
    }
    if (!bra_io_file_write(dst, &chunk_header->huffman, sizeof(bra_huffman_t)))
    {
        bra_log_error("unable to write chunk huffman header to %s", dst->fn);
        return false;
    }
    return true;
}

bool bra_io_file_chunks_read_file(bra_io_file_t* src, const uint64_t data_size, bra_meta_entry_t* me, const bool decode)
{
    assert(src != NULL && me != NULL);
    const unsigned comp = BRA_ATTR_COMP(me->attributes);
    if (comp == BRA_ATTR_COMP_STORED)
        return bra_io_file_chunks_copy_file(NULL, src, data_size, me, decode);
    if (comp == BRA_ATTR_COMP_COMPRESSED)
        return bra_io_file_chunks_decompress_file(NULL, src, data_size, me, decode);
    bra_log_critical("invalid compression type for file: %u", comp);
    return false;
}

/* Stored data: copied through in CHUNK_SIZE pieces, the CRC updated per piece (:119-167). */
bool bra_io_file_chunks_copy_file(bra_io_file_t* dst, bra_io_file_t* src, const uint64_t data_size, bra_meta_entry_t* me, const bool compute_crc32)
{
    assert(src != NULL);
    bool     ok  = !(dst != NULL && (dst->f == NULL || dst->fn == NULL));
    uint8_t* buf = ok ? (uint8_t*) malloc(CHUNK_SIZE) : NULL;
    if (ok && compute_crc32 && me == NULL)
    {
        bra_log_critical("can't compute crc32: me is null");
        ok = false;
    }
    for (uint64_t done = 0; ok && buf != NULL && done < data_size;)
    {
        const size_t n = (size_t) _bra_min(CHUNK_SIZE, data_size - done);
        ok             = bra_io_file_read(src, buf, n);
        if (ok && compute_crc32)
            me->crc32 = bra_crc32c(buf, n, me->crc32);
        if (ok && dst != NULL)
            ok = bra_io_file_write(dst, buf, n);
        done += n;
    }
    ok = ok && buf != NULL;
    free(buf);
    if (!ok)
    {
        if (dst != NULL)
            bra_io_file_close(dst);
        bra_io_file_close(src);
    }
    return ok;
}

static uint64_t num_chunks(uint64_t n) { return (n + CHUNK_SIZE - 1) / CHUNK_SIZE; }

/* A batch read from the source file on a helper thread, so that reading batch k + 2 overlaps the
 * device work of batches k and k + 1 (the reference reads, encodes and writes one chunk after the
 * other, lib_bra_io_file_chunks.c:199-266). */
typedef struct
{
    bra_io_file_t* src;
    uint8_t*       buf;
    uint64_t       n;
    bool           ok;
    pthread_t      th;
    bool           running;
} batch_read_t;

static void* batch_read_main(void* arg)
{
    batch_read_t* r = (batch_read_t*) arg;
    r->ok           = bra_io_file_read(r->src, r->buf, r->n);
    return NULL;
}

static void batch_read_start(batch_read_t* r, bra_io_file_t* src, uint8_t* buf, uint64_t n)
{
    r->src = src, r->buf = buf, r->n = n, r->ok = false;
    r->running = pthread_create(&r->th, NULL, batch_read_main, r) == 0;
    if (!r->running)
        r->ok = bra_io_file_read(src, buf, n); /* no thread: read inline */
}

static bool batch_read_join(batch_read_t* r)
{
    if (r->running)
        pthread_join(r->th, NULL);
    r->running = false;
    return r->ok;
}

bool bra_io_file_chunks_compress_file(bra_io_file_t* dst, bra_io_file_t* src, const uint64_t data_size, bra_meta_entry_t* me)
{
    assert(dst != NULL && src != NULL && me != NULL);
    bra_gpu_ctx_t* ctx = front_ctx();
    if (ctx == NULL)
        return false;
    // the records of the compressed chunks go to a temporary file first: kept only when smaller
    // than the input (the reference's rule, :185-189 and :268-278)
    bra_io_file_t tmpfile;
    if (!bra_io_file_tmp_open(&tmpfile))
    {
        bra_log_error("unable to compress file: %s", src->fn);
        return false;
    }
    // Batches of BATCH_CHUNKS chunks, two in flight on the device (bra_gpu_compress_chunks_stage /
    // _submit / _collect): batch k + 1's input copy is queued before batch k is submitted, so it
    // arrives while batch k's kernels run; batch k - 1's records are copied back and written while
    // batch k's later stages run; batch k + 2 is read from the file meanwhile.  Pinned host buffers
    // make the copies asynchronous.
    const uint64_t batch  = _bra_min((uint64_t) BATCH_CHUNKS * CHUNK_SIZE, data_size);
    const uint64_t nbatch = batch ? (data_size + batch - 1) / batch : 0;
    const uint64_t cap    = bra_gpu_chunks_bound(batch, (uint32_t) CHUNK_SIZE);
    uint8_t*       in[2]  = {(uint8_t*) bra_gpu_host_alloc(ctx, batch ? batch : 1), (uint8_t*) bra_gpu_host_alloc(ctx, batch ? batch : 1)};
    uint8_t*       out    = (uint8_t*) bra_gpu_host_alloc(ctx, cap ? cap : 1);
    uint32_t       crc32  = BRA_CRC32C_INIT; /* the running CRC of header + source chunk pairs (:214,248-249) */
    bool           ok     = in[0] != NULL && in[1] != NULL && out != NULL;
    bool           read_failed = false;
    batch_read_t   rd;
    memset(&rd, 0, sizeof rd);
#define BATCH_LEN(k) _bra_min(batch, data_size - (uint64_t) (k) * batch)
#define STAGE(k) (bra_gpu_compress_chunks_stage(ctx, (int) ((k) % 2), in[(k) % 2], BATCH_LEN(k)) == 0)
    if (ok && nbatch > 0)
    {
        read_failed = !bra_io_file_read(src, in[0], BATCH_LEN(0));
        ok          = !read_failed && STAGE(0);
        if (ok && nbatch > 1)
            batch_read_start(&rd, src, in[1], BATCH_LEN(1));
    }
    for (uint64_t k = 0; ok && k <= nbatch; ++k)
    {
        if (k < nbatch)
        {
            bra_log_printf("%3u%%", (unsigned int) (k * batch * 100 / data_size));
            bra_log_printf("\b\b\b\b");
            // batch k + 1 (read into in[(k + 1) % 2]) is staged ahead of batch k's submit -- after it
            // for the first batch, which goes to the device before the second one has been read
            const bool stage_ahead = k > 0 && k + 1 < nbatch;
            if (stage_ahead && !(read_failed = !batch_read_join(&rd)) && !STAGE(k + 1))
                ok = false;
            if (read_failed || !ok)
                break;
            if (bra_gpu_compress_chunks_submit(ctx, (int) (k % 2), in[k % 2], BATCH_LEN(k), (uint32_t) CHUNK_SIZE) != 0)
            {
                bra_log_error("GPU chunk encoder failed: %s (chunks from %" PRIu64 ")", src->fn, k * batch);
                ok = false;
                break;
            }
            if (k == 0 && nbatch > 1 && !(read_failed = !batch_read_join(&rd)) && !STAGE(1))
                ok = false;
            if (read_failed || !ok)
                break;
            // in[k % 2] is free once batch k's submit has returned: batch k + 2 is read into it
            if (k + 2 < nbatch)
                batch_read_start(&rd, src, in[k % 2], BATCH_LEN(k + 2));
        }
        if (k == 0)
            continue;
        uint64_t osz  = 0;
        uint32_t bcrc = 0;
        if (bra_gpu_compress_chunks_collect(ctx, (int) ((k - 1) % 2), out, cap, &osz, &bcrc) < 0)
        {
            bra_log_error("GPU chunk encoder failed: %s (chunks from %" PRIu64 ")", src->fn, (k - 1) * batch);
            ok = false;
            break;
        }
        // this batch's share of the running CRC: its headers and chunks follow the previous ones
        const uint64_t n = BATCH_LEN(k - 1);
        crc32 = bra_gpu_crc32c_combine(crc32, bcrc, n + num_chunks(n) * sizeof(bra_io_chunk_header_t));
        ok    = bra_io_file_write(&tmpfile, out, (size_t) osz);
    }
#undef STAGE
#undef BATCH_LEN
    (void) batch_read_join(&rd);
    if (read_failed || !ok)
        for (int q = 0; q < 2; ++q)  // batches still in flight or staged after an error: drained, dropped
            (void) bra_gpu_compress_chunks_collect(ctx, q, NULL, 0, NULL, NULL);
    bra_gpu_host_free(ctx, in[0]);
    bra_gpu_host_free(ctx, in[1]);
    bra_gpu_host_free(ctx, out);
    if (read_failed)
    {
        // the reference's read-error path (:203-210): tmpfile and dst closed, the caller closes src
        bra_io_file_close(&tmpfile);
        bra_io_file_close(dst);
        return false;
    }
    if (!ok)
    {
        bra_io_file_close(&tmpfile);
        bra_io_file_close(dst);
        bra_io_file_close(src);
        return false;
    }

    const int64_t tmpfile_size = bra_io_file_tell(&tmpfile);
    bool          res          = tmpfile_size >= 0;
    if (res && (uint64_t) tmpfile_size >= data_size)
    {
        res            = false; /* not smaller: the caller stores the file instead */
        me->attributes = BRA_ATTR_SET_COMP(me->attributes, BRA_ATTR_COMP_STORED);
    }
    else if (res)
    {
        bra_meta_entry_file_t* mef = (bra_meta_entry_file_t*) me->entry_data;
        mef->data_size             = (uint64_t) tmpfile_size;
        me->crc32                  = bra_crc32c(&tmpfile_size, sizeof(tmpfile_size), me->crc32);
        me->crc32                  = bra_crc32c_combine(me->crc32, crc32, data_size + (num_chunks(data_size) * sizeof(bra_io_chunk_header_t)));
        res = bra_io_file_seek(&tmpfile, 0, SEEK_SET) && bra_io_file_meta_entry_write_file_entry(dst, me) &&
              bra_io_file_chunks_copy_file(dst, &tmpfile, (uint64_t) tmpfile_size, me, false);
    }
    bra_io_file_close(&tmpfile);
    return res;
}

/* Header checks of the reference decoder (:31-49). */
static bool header_valid(const bra_io_chunk_header_t* h)
{
    return h->primary_index < BRA_MAX_CHUNK_SIZE && h->huffman.encoded_size <= BRA_MAX_CHUNK_SIZE &&
           h->huffman.orig_size <= BRA_MAX_CHUNK_SIZE && h->huffman.encoded_size != 0 && h->huffman.orig_size != 0;
}

/* Listing (decode == false): only the decoded sizes, through the per-chunk entry points. */
static bool chunk_decoded_size(const bra_io_chunk_header_t* h, const uint8_t* payload, uint64_t* size)
{
    uint32_t       huf_s = 0;
    uint8_t* const huf   = bra_huffman_decode(&h->huffman, payload, &huf_s);
    if (huf == NULL)
        return false;
    *size += bra_rle_decode_compute_size(huf, huf_s);
    free(huf);
    return true;
}

/* The records [0, recs) of a batch decoded one at a time through the per-chunk entry points (the
 * reference's loop body, :355-405): dst receives every chunk before the first bad one, and the
 * failure is logged with the reference's message.  Used only after the batched decode failed.
 * tmp holds 2 * CHUNK_SIZE bytes. */
static bool decode_records_serial(bra_io_file_t* dst, const char* fn, const uint8_t* stream, uint32_t recs, bra_meta_entry_t* me, uint64_t* orig,
                                  uint8_t* tmp)
{
    const uint64_t hsz = BRA_BWT_INDEX_BYTES + sizeof(bra_huffman_t);
    uint64_t       p   = 0;
    for (uint32_t r = 0; r < recs; ++r)
    {
        bra_io_chunk_header_t h = {.primary_index = 0};
        h.primary_index         = (bra_bwt_index_t) stream[p] | (bra_bwt_index_t) stream[p + 1] << 8 | (bra_bwt_index_t) stream[p + 2] << 16;
        memcpy(&h.huffman, stream + p + BRA_BWT_INDEX_BYTES, sizeof(bra_huffman_t));
        uint32_t       huf_s = 0;
        uint8_t* const huf   = bra_huffman_decode(&h.huffman, stream + p + hsz, &huf_s);
        if (huf == NULL)
        {
            bra_log_error("unable to decode huffman file: %s ", fn);
            return false;
        }
        uint8_t*   rle = NULL;
        size_t     s   = 0;
        const bool rok = bra_rle_decode(huf, huf_s, &rle, &s);
        free(huf);
        if (!rok)
        {
            bra_log_error("unable to decode RLE in %s", fn);
            return false;
        }
        *orig += s;
        if (s > CHUNK_SIZE)
        {
            // no reference equivalent: the reference decodes into its 256 KiB g_buf without this
            // check; here it protects the tmp buffer
            bra_log_error("decoded chunk size %zu exceeds BRA_MAX_CHUNK_SIZE in %s", s, fn);
            free(rle);
            return false;
        }
        if (h.primary_index >= s)
        {
            bra_log_error("invalid primary index (%u) for chunk size %zu in %s", h.primary_index, s, fn);
            free(rle);
            return false;
        }
        bra_mtf_decode2(rle, s, tmp);
        free(rle);
        bra_bwt_decode2(tmp, (bra_bwt_index_t) s, h.primary_index, NULL, tmp + CHUNK_SIZE);
        me->crc32 = bra_crc32c(&h, sizeof(bra_io_chunk_header_t), me->crc32);
        me->crc32 = bra_crc32c(tmp + CHUNK_SIZE, s, me->crc32);
        if (dst != NULL && !bra_io_file_write(dst, tmp + CHUNK_SIZE, s))
            return false;
        p += hsz + h.huffman.encoded_size;
    }
    return true;
}

bool bra_io_file_chunks_decompress_file(bra_io_file_t* dst, bra_io_file_t* src, const uint64_t data_size, bra_meta_entry_t* me, const bool decode)
{
    assert(src != NULL && me != NULL);
    bra_gpu_ctx_t* ctx = decode ? front_ctx() : NULL;
    bool           ok  = !(dst != NULL && (dst->f == NULL || dst->fn == NULL)) && (!decode || ctx != NULL);
    // a batch holds whole records: up to BATCH_CHUNKS of them, at most that many chunk sizes of
    // decoded output (the headers bound every chunk by BRA_MAX_CHUNK_SIZE)
    const uint64_t rec_max  = sizeof(bra_huffman_t) + BRA_BWT_INDEX_BYTES + CHUNK_SIZE;
    const uint64_t scap     = (uint64_t) BATCH_CHUNKS * rec_max;
    const uint64_t ocap     = (uint64_t) (BATCH_CHUNKS < 2 ? 2 : BATCH_CHUNKS) * CHUNK_SIZE;
    uint8_t*       stream   = ok ? (uint8_t*) malloc(scap) : NULL;
    uint8_t*       decoded  = (ok && decode) ? (uint8_t*) malloc(ocap) : NULL;
    uint64_t       orig     = 0;
    ok                      = ok && stream != NULL && (!decode || decoded != NULL);
    for (uint64_t done = 0; ok && done < data_size;)
    {
        // read up to BATCH_CHUNKS records (header, check, payload) into the stream buffer; a bad
        // header or a failed read ends the batch after the good records before it
        uint64_t fill = 0;
        uint32_t recs = 0;
        bool     bad  = false;
        while (!bad && recs < BATCH_CHUNKS && done + fill < data_size)
        {
            bra_io_chunk_header_t h = {.primary_index = 0};
            bad = !bra_io_file_chunks_read_header(src, &h);
            if (!bad && !header_valid(&h))
            {
                bra_log_error("chunk header not valid in %s", src->fn);
                bad = true;
            }
            if (bad)
                break;
            uint8_t* rec = stream + fill;
            rec[0] = (uint8_t) h.primary_index, rec[1] = (uint8_t) (h.primary_index >> 8), rec[2] = (uint8_t) (h.primary_index >> 16);
            memcpy(rec + BRA_BWT_INDEX_BYTES, &h.huffman, sizeof(bra_huffman_t));
            const uint64_t hsz = BRA_BWT_INDEX_BYTES + sizeof(bra_huffman_t);
            bad                = !bra_io_file_read(src, rec + hsz, h.huffman.encoded_size);
            if (!bad && !decode && !chunk_decoded_size(&h, rec + hsz, &orig))
            {
                bra_log_error("unable to decode huffman file: %s ", src->fn);
                bad = true;
            }
            if (bad)
                break;
            fill += hsz + h.huffman.encoded_size;
            ++recs;
        }
        if (decode && recs > 0)
        {
            // the reference writes every chunk before a bad record: decode the good ones first
            uint64_t  osz = 0;
            uint32_t  crc = me->crc32;
            const int rc  = bad ? -1 : bra_gpu_decompress_chunks_host(ctx, stream, fill, (uint32_t) CHUNK_SIZE, decoded, ocap, &osz, me->crc32, &crc, 0);
            if (rc == 0)
            {
                me->crc32 = crc;
                orig += osz;
                if (dst != NULL)
                    ok = bra_io_file_write(dst, decoded, (size_t) osz);
            }
            else
                ok = decode_records_serial(dst, src->fn, stream, recs, me, &orig, decoded) && !bad;
        }
        ok = ok && !bad;
        done += fill;
    }
    if (ok && orig <= data_size)
    {
        bra_log_error("corrupted file entry: %s", me->name);
        ok = false;
    }
    if (ok)
        me->_compression_ratio = (float) ((double) data_size / (double) orig);
    free(stream);
    free(decoded);
    if (!ok)
    {
        if (dst != NULL)
            bra_io_file_close(dst);
        bra_io_file_close(src);
    }
    return ok;
}
