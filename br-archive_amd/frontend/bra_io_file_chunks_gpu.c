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
#include <errno.h>
#include <sys/stat.h>
#include <unistd.h>
#include <time.h>
#include <sys/mman.h>

#define CHUNK_SIZE ((uint64_t) BRA_MAX_CHUNK_SIZE)
#ifndef BATCH_CHUNKS
#define BATCH_CHUNKS 256u /* 64 MiB of input per device call (tests build a 2-chunk variant) */
#endif

/* BRA_FRONT_TIMING=1: a per-file breakdown of the chunk loops' wall clock on stderr (measurement). */
static int front_timing(void)
{
    static int t = -1;
    if (t < 0)
    {
        const char* e = getenv("BRA_FRONT_TIMING");
        t             = (e != NULL && e[0] == '1') ? 1 : 0;
    }
    return t;
}
static double now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* load time of this library (a timestamp only: no device call), for the breakdown above */
static double g_t_load;
__attribute__((constructor)) static void front_loaded(void) { g_t_load = now_ms(); }

/* One device context for the front end, created once (pthread_once) on the device current when
 * lib_bra first compresses or decompresses, and destroyed at process exit, with the pinned batch
 * buffers that it keeps for every file (grown when a larger batch needs them). */
static bra_gpu_ctx_t*  g_front_ctx  = NULL;
static pthread_once_t  g_front_once = PTHREAD_ONCE_INIT;

typedef struct
{
    uint8_t* in[2];  /* pinned input batches */
    uint64_t cap_in;
    uint8_t* out;  /* pinned chunk records of one batch */
    uint64_t cap_out;
    uint8_t* rec;  /* a file's chunk records kept in memory (malloc) instead of the tmpfile */
    uint64_t cap_rec;
} front_bufs_t;
static front_bufs_t g_fb;
static void         rec_free(uint8_t* p, uint64_t bytes);
static void         front_dec_release(void);

static void front_bufs_release(void)
{
    for (int q = 0; q < 2; ++q)
        bra_gpu_host_free(g_front_ctx, g_fb.in[q]);
    bra_gpu_host_free(g_front_ctx, g_fb.out);
    rec_free(g_fb.rec, g_fb.cap_rec);
    memset(&g_fb, 0, sizeof g_fb);
}

static void front_ctx_destroy(void)
{
    const double t = front_timing() ? now_ms() : 0;
    front_bufs_release();
    front_dec_release();
    bra_gpu_ctx_destroy(g_front_ctx);
    g_front_ctx = NULL;
    if (front_timing())
        fprintf(stderr, "front: context and buffers released at exit in %.1f ms\n", now_ms() - t);
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

/* The pinned buffers for batches of `batch` bytes (kept across files; grown, never shrunk). */
static bool front_bufs(bra_gpu_ctx_t* ctx, uint64_t batch)
{
    const uint64_t rb = bra_gpu_pipe_records_bound(batch, (uint32_t) BRA_MAX_CHUNK_SIZE);
    if (batch > g_fb.cap_in)
    {
        for (int q = 0; q < 2; ++q)
        {
            bra_gpu_host_free(ctx, g_fb.in[q]);
            g_fb.in[q] = (uint8_t*) bra_gpu_host_alloc(ctx, batch);
        }
        g_fb.cap_in = (g_fb.in[0] != NULL && g_fb.in[1] != NULL) ? batch : 0;
    }
    if (rb > g_fb.cap_out)
    {
        bra_gpu_host_free(ctx, g_fb.out);
        g_fb.out     = (uint8_t*) bra_gpu_host_alloc(ctx, rb);
        g_fb.cap_out = g_fb.out != NULL ? rb : 0;
    }
    return g_fb.cap_in >= batch && g_fb.cap_out >= rb;
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

/* Batches are read from the source file on a helper thread, so that reading batch k + 2 overlaps
 * the device work of batches k and k + 1 (the reference reads, encodes and writes one chunk after
 * the other, lib_bra_io_file_chunks.c:199-266).  A regular file is read with positioned reads
 * (pread) on READ_THREADS threads at once -- one thread's copies out of the page cache are slower
 * than the device encodes -- and the FILE's position is set past the data at the end, as the
 * reference's sequential freads leave it.  Other files are read with bra_io_file_read. */
#ifndef READ_THREADS
#define READ_THREADS 4
#endif
#define READ_PIECE ((uint64_t) 4 << 20)

typedef struct
{
    int      fd;
    uint8_t* buf;
    uint64_t n;
    int64_t  off;
    int      err; /* errno of a failed read, -1 for a short one */
} read_piece_t;

static void* read_piece_main(void* arg)
{
    read_piece_t* p = (read_piece_t*) arg;
    for (uint64_t done = 0; done < p->n;)
    {
        const ssize_t r = pread(p->fd, p->buf + done, (size_t) (p->n - done), (off_t) (p->off + (int64_t) done));
        if (r < 0 && errno == EINTR)
            continue;
        if (r <= 0)
        {
            p->err = r < 0 ? errno : -1;
            return NULL;
        }
        done += (uint64_t) r;
    }
    return NULL;
}

typedef struct
{
    bra_io_file_t* src;
    int            fd;  /* >= 0: positioned reads from file offset `off` */
    int64_t        off;
    uint8_t*       buf;
    uint64_t       n;
    bool           ok;
    int            err;
    pthread_t      th;
    bool           running;
} batch_read_t;

static void batch_read_run(batch_read_t* r)
{
    if (r->fd < 0)
    {
        r->ok = bra_io_file_read(r->src, r->buf, r->n);
        return;
    }
    read_piece_t p[READ_THREADS];
    pthread_t    th[READ_THREADS];
    bool         started[READ_THREADS] = {false};
    const uint64_t per = ((r->n + READ_THREADS - 1) / READ_THREADS + READ_PIECE - 1) / READ_PIECE * READ_PIECE;
    int          np  = 0;
    for (uint64_t o = 0; o < r->n && np < READ_THREADS; o += per, ++np)
        p[np] = (read_piece_t){.fd = r->fd, .buf = r->buf + o, .n = _bra_min(per, r->n - o), .off = r->off + (int64_t) o, .err = 0};
    for (int i = 1; i < np; ++i)
        started[i] = pthread_create(&th[i], NULL, read_piece_main, &p[i]) == 0;
    read_piece_main(&p[0]);
    for (int i = 1; i < np; ++i)
        if (started[i])
            pthread_join(th[i], NULL);
        else
            read_piece_main(&p[i]);
    r->ok  = true;
    r->err = 0;
    for (int i = 0; i < np; ++i)
        if (p[i].err != 0)
        {
            r->ok  = false;
            r->err = p[i].err;
            break;
        }
}

static void* batch_read_main(void* arg)
{
    batch_read_run((batch_read_t*) arg);
    return NULL;
}

static void batch_read_start(batch_read_t* r, uint8_t* buf, uint64_t n, int64_t off)
{
    r->buf = buf, r->n = n, r->off = off, r->ok = false, r->err = 0;
    r->running = pthread_create(&r->th, NULL, batch_read_main, r) == 0;
    if (!r->running)
        batch_read_run(r); /* no thread: read inline */
}

/* Joins the read; on a failed positioned read reports it as the reference's bra_io_file_read does
 * (logged, src closed) -- on the calling thread, after the join. */
static bool batch_read_join(batch_read_t* r)
{
    if (r->running)
        pthread_join(r->th, NULL);
    r->running = false;
    if (!r->ok && r->fd >= 0 && r->src->f != NULL)
    {
        errno = r->err > 0 ? r->err : 0;
        bra_io_file_read_error(r->src);
    }
    return r->ok;
}

/* The chunk records of one file: in memory (g_fb.rec) while they stay below REC_MEM_MAX bytes, then
 * spilled to a temporary file as the reference writes them (:185-189). */
#ifndef REC_MEM_MAX
#define REC_MEM_MAX ((uint64_t) 1 << 30)
#endif
typedef struct
{
    uint64_t      len;
    bool          spilled;
    bra_io_file_t tmp;
} records_t;

/* Anonymous memory with transparent huge pages where the kernel allows them: the records of a large
 * file are written once into fresh pages, and 4 KiB page faults cost more than the copy. */
static uint8_t* rec_alloc(uint64_t bytes)
{
    void* p = mmap(NULL, (size_t) bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED)
        return NULL;
#ifdef MADV_HUGEPAGE
    (void) madvise(p, (size_t) bytes, MADV_HUGEPAGE);
#endif
    return (uint8_t*) p;
}

static void rec_free(uint8_t* p, uint64_t bytes)
{
    if (p != NULL)
        (void) munmap(p, (size_t) bytes);
}

static bool records_put(records_t* rs, const uint8_t* p, uint64_t n)
{
    if (!rs->spilled && rs->len + n <= REC_MEM_MAX)
    {
        if (rs->len + n > g_fb.cap_rec)
        {
            uint64_t cap = g_fb.cap_rec ? g_fb.cap_rec : ((uint64_t) 64 << 20);
            while (cap < rs->len + n)
                cap *= 2;
            uint8_t* q = rec_alloc(cap);
            if (q == NULL)
                goto spill;
            if (rs->len > 0)
                memcpy(q, g_fb.rec, rs->len);
            rec_free(g_fb.rec, g_fb.cap_rec);
            g_fb.rec = q, g_fb.cap_rec = cap;
        }
        memcpy(g_fb.rec + rs->len, p, n);
        rs->len += n;
        return true;
    }
spill:
    if (!rs->spilled)
    {
        memset(&rs->tmp, 0, sizeof rs->tmp);
        if (!bra_io_file_tmp_open(&rs->tmp))
            return false;
        rs->spilled = true;
        if (rs->len > 0 && !bra_io_file_write(&rs->tmp, g_fb.rec, (size_t) rs->len))
            return false;
    }
    rs->len += n;
    return bra_io_file_write(&rs->tmp, p, (size_t) n);
}

/* Address space for a file's records up front (pages are only touched as records arrive), so the
 * buffer does not move while it fills. */
static void records_reserve(uint64_t bytes)
{
    bytes = _bra_min(bytes, REC_MEM_MAX);
    if (bytes <= g_fb.cap_rec)
        return;
    uint8_t* q = rec_alloc(bytes);
    if (q == NULL)
        return;  // records_put grows it (or spills) as needed
    rec_free(g_fb.rec, g_fb.cap_rec);
    g_fb.rec = q, g_fb.cap_rec = bytes;
}

static void records_close(records_t* rs)
{
    if (rs->spilled && rs->tmp.f != NULL)
        bra_io_file_close(&rs->tmp);
}

bool bra_io_file_chunks_compress_file(bra_io_file_t* dst, bra_io_file_t* src, const uint64_t data_size, bra_meta_entry_t* me)
{
    assert(dst != NULL && src != NULL && me != NULL);
    const int    tm = front_timing();
    const double t0 = tm ? now_ms() : 0;
    double       t_read = 0, t_submit = 0, t_collect = 0, t_rec = 0, t_ctx = 0;
    double       tt;
#define TICK() (tt = tm ? now_ms() : 0)
#define TOCK(acc) (acc += tm ? now_ms() - tt : 0)
    // Batches of BATCH_CHUNKS chunks, two in flight on the device (bra_gpu_compress_chunks_stage /
    // _submit / _collect): batch k + 1's input copy is queued before batch k is submitted, so it
    // arrives while batch k's kernels run; batch k - 1's records are copied back and kept while
    // batch k's later stages run; batch k + 2 is read from the file meanwhile.  Pinned host buffers
    // (kept with the context across files) make the copies asynchronous.
    const uint64_t batch  = _bra_min((uint64_t) BATCH_CHUNKS * CHUNK_SIZE, data_size);
    const uint64_t nbatch = batch ? (data_size + batch - 1) / batch : 0;
    if (tm && g_front_ctx == NULL)
        fprintf(stderr, "front: first chunk loop call %.1f ms after the library was loaded\n", t0 - g_t_load);
    TICK();
    bra_gpu_ctx_t* ctx = front_ctx();
    TOCK(t_ctx);
    double t_bufs = 0;
    TICK();
    bool ok = ctx != NULL && front_bufs(ctx, batch ? batch : 1);
    TOCK(t_bufs);
    if (ctx == NULL)
        return false;
    // the records of the compressed chunks are collected first (in memory, or in a temporary file
    // beyond REC_MEM_MAX): kept only when smaller than the input (the reference's rule, :185-189 and
    // :268-278)
    records_t rs;
    memset(&rs, 0, sizeof rs);
    records_reserve(bra_gpu_pipe_records_bound(data_size, (uint32_t) CHUNK_SIZE));
    uint8_t** in          = g_fb.in;
    uint8_t*  out         = g_fb.out;
    uint32_t  crc32       = BRA_CRC32C_INIT; /* the running CRC of header + source chunk pairs (:214,248-249) */
    bool      read_failed = false;
    // positioned reads when src is a regular file (its FILE position is then restored at the end)
    struct stat st;
    const int     fd0   = fileno(src->f);
    const int64_t pos0  = bra_io_file_tell(src);
    batch_read_t  rd;
    memset(&rd, 0, sizeof rd);
    rd.src = src;
    rd.fd  = (fd0 >= 0 && pos0 >= 0 && fstat(fd0, &st) == 0 && S_ISREG(st.st_mode)) ? fd0 : -1;
    if (!ok)
        bra_log_error("unable to compress file: %s", src->fn);
#define BATCH_LEN(k) _bra_min(batch, data_size - (uint64_t) (k) * batch)
#define BATCH_OFF(k) (pos0 + (int64_t) ((uint64_t) (k) * batch))
#define STAGE(k) (bra_gpu_compress_chunks_stage(ctx, (int) ((k) % 2), in[(k) % 2], BATCH_LEN(k)) == 0)
    if (ok && nbatch > 0)
    {
        TICK();
        batch_read_start(&rd, in[0], BATCH_LEN(0), BATCH_OFF(0));
        read_failed = !batch_read_join(&rd);
        TOCK(t_read);
        ok = !read_failed && STAGE(0);
        if (ok && nbatch > 1)
            batch_read_start(&rd, in[1], BATCH_LEN(1), BATCH_OFF(1));
    }
    uint64_t fail_at = UINT64_MAX;  // the first chunk of a batch the device failed on
    for (uint64_t k = 0; ok && k <= nbatch; ++k)
    {
        if (k < nbatch)
        {
            bra_log_printf("%3u%%", (unsigned int) (k * batch * 100 / data_size));
            bra_log_printf("\b\b\b\b");
            // batch k + 1 (read into in[(k + 1) % 2]) is staged ahead of batch k's submit -- after it
            // for the first batch, which goes to the device before the second one has been read
            const bool stage_ahead = k > 0 && k + 1 < nbatch;
            TICK();
            if (stage_ahead && !(read_failed = !batch_read_join(&rd)) && !STAGE(k + 1))
                ok = false;
            TOCK(t_read);
            if (read_failed || !ok)
                break;
            TICK();
            if (bra_gpu_compress_chunks_submit(ctx, (int) (k % 2), in[k % 2], BATCH_LEN(k), (uint32_t) CHUNK_SIZE) != 0)
            {
                fail_at = k * batch;
                ok      = false;
                break;
            }
            TOCK(t_submit);
            TICK();
            if (k == 0 && nbatch > 1 && !(read_failed = !batch_read_join(&rd)) && !STAGE(1))
                ok = false;
            TOCK(t_read);
            if (read_failed || !ok)
                break;
            // in[k % 2] is free once batch k's submit has returned: batch k + 2 is read into it
            if (k + 2 < nbatch)
                batch_read_start(&rd, in[k % 2], BATCH_LEN(k + 2), BATCH_OFF(k + 2));
        }
        if (k == 0)
            continue;
        uint64_t osz  = 0;
        uint32_t bcrc = 0;
        TICK();
        if (bra_gpu_compress_chunks_collect(ctx, (int) ((k - 1) % 2), out, g_fb.cap_out, &osz, &bcrc) < 0)
        {
            fail_at = (k - 1) * batch;
            ok      = false;
            break;
        }
        TOCK(t_collect);
        // this batch's share of the running CRC: its headers and chunks follow the previous ones
        const uint64_t n = BATCH_LEN(k - 1);
        crc32 = bra_gpu_crc32c_combine(crc32, bcrc, n + num_chunks(n) * sizeof(bra_io_chunk_header_t));
        TICK();
        ok = records_put(&rs, out, osz);
        TOCK(t_rec);
    }
#undef STAGE
#undef BATCH_OFF
#undef BATCH_LEN
    // the reader is joined before src is used again (a failed read closes it)
    if (rd.running && !batch_read_join(&rd))
        read_failed = true;
    if (fail_at != UINT64_MAX)
        bra_log_error("GPU chunk encoder failed: %s (chunks from %" PRIu64 ")", src->f != NULL ? src->fn : "N/A", fail_at);
    if (read_failed || !ok)
        for (int q = 0; q < 2; ++q)  // batches still in flight or staged after an error: drained, dropped
            (void) bra_gpu_compress_chunks_collect(ctx, q, NULL, 0, NULL, NULL);
    if (rd.fd >= 0 && !read_failed && ok && !bra_io_file_seek(src, pos0 + (int64_t) data_size, SEEK_SET))
        ok = false;
    if (read_failed)
    {
        // the reference's read-error path (:203-210): tmpfile and dst closed, the caller closes src
        records_close(&rs);
        bra_io_file_close(dst);
        return false;
    }
    if (!ok)
    {
        records_close(&rs);
        bra_io_file_close(dst);
        if (src->f != NULL)
            bra_io_file_close(src);
        return false;
    }

    TICK();
    const int64_t rec_size = (int64_t) rs.len;
    bool          res      = true;
    if ((uint64_t) rec_size >= data_size)
    {
        res            = false; /* not smaller: the caller stores the file instead */
        me->attributes = BRA_ATTR_SET_COMP(me->attributes, BRA_ATTR_COMP_STORED);
    }
    else
    {
        bra_meta_entry_file_t* mef = (bra_meta_entry_file_t*) me->entry_data;
        mef->data_size             = (uint64_t) rec_size;
        me->crc32                  = bra_crc32c(&rec_size, sizeof(rec_size), me->crc32);
        me->crc32                  = bra_crc32c_combine(me->crc32, crc32, data_size + (num_chunks(data_size) * sizeof(bra_io_chunk_header_t)));
        res = bra_io_file_meta_entry_write_file_entry(dst, me);
        if (res && rs.spilled)
            res = bra_io_file_seek(&rs.tmp, 0, SEEK_SET) && bra_io_file_chunks_copy_file(dst, &rs.tmp, (uint64_t) rec_size, me, false);
        else if (res && rec_size > 0)
            res = bra_io_file_write(dst, g_fb.rec, (size_t) rec_size);
    }
    records_close(&rs);
    double t_out = 0;
    TOCK(t_out);
    if (tm)
        fprintf(stderr,
                "front: compress %" PRIu64 " bytes in %.1f ms: ctx %.1f, pinned buffers %.1f, read waits %.1f, submit %.1f, collect %.1f, records %.1f, "
                "archive write %.1f (records %" PRIu64 " bytes, %s)\n",
                data_size, now_ms() - t0, t_ctx, t_bufs, t_read, t_submit, t_collect, t_rec, t_out, (uint64_t) rec_size,
                rs.spilled ? "spilled to tmpfile" : "in memory");
#undef TICK
#undef TOCK
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
    // the reference contract of bra_bwt_decode2 asks for a transform buffer (bra_bwt.c:137)
    bra_bwt_index_t* trans = (bra_bwt_index_t*) malloc(CHUNK_SIZE * sizeof(bra_bwt_index_t));
    if (trans == NULL)
        return false;
    bool ok = true;
    for (uint32_t r = 0; ok && r < recs; ++r)
    {
        bra_io_chunk_header_t h = {.primary_index = 0};
        h.primary_index         = (bra_bwt_index_t) stream[p] | (bra_bwt_index_t) stream[p + 1] << 8 | (bra_bwt_index_t) stream[p + 2] << 16;
        memcpy(&h.huffman, stream + p + BRA_BWT_INDEX_BYTES, sizeof(bra_huffman_t));
        uint32_t       huf_s = 0;
        uint8_t* const huf   = bra_huffman_decode(&h.huffman, stream + p + hsz, &huf_s);
        if (huf == NULL)
        {
            bra_log_error("unable to decode huffman file: %s ", fn);
            ok = false;
            break;
        }
        uint8_t*   rle = NULL;
        size_t     s   = 0;
        const bool rok = bra_rle_decode(huf, huf_s, &rle, &s);
        free(huf);
        if (!rok)
        {
            bra_log_error("unable to decode RLE in %s", fn);
            ok = false;
            break;
        }
        *orig += s;
        if (s > CHUNK_SIZE)
        {
            // no reference equivalent: the reference decodes into its 256 KiB g_buf without this
            // check; here it protects the tmp buffer
            bra_log_error("decoded chunk size %zu exceeds BRA_MAX_CHUNK_SIZE in %s", s, fn);
            free(rle);
            ok = false;
            break;
        }
        if (h.primary_index >= s)
        {
            bra_log_error("invalid primary index (%u) for chunk size %zu in %s", h.primary_index, s, fn);
            free(rle);
            ok = false;
            break;
        }
        bra_mtf_decode2(rle, s, tmp);
        free(rle);
        bra_bwt_decode2(tmp, (bra_bwt_index_t) s, h.primary_index, trans, tmp + CHUNK_SIZE);
        me->crc32 = bra_crc32c(&h, sizeof(bra_io_chunk_header_t), me->crc32);
        me->crc32 = bra_crc32c(tmp + CHUNK_SIZE, s, me->crc32);
        if (dst != NULL && !bra_io_file_write(dst, tmp + CHUNK_SIZE, s))
        {
            ok = false;
            break;
        }
        p += hsz + h.huffman.encoded_size;
    }
    free(trans);
    return ok;
}

/* The decoded output of batch k is written to dst on a helper thread while batch k + 1 is read and
 * decoded (the reference decodes and writes one chunk after the other, :355-405). */
typedef struct
{
    bra_io_file_t* dst;
    const uint8_t* buf;
    uint64_t       n;
    bool           ok;
    pthread_t      th;
    bool           running;
} batch_write_t;

static void* batch_write_main(void* arg)
{
    batch_write_t* w = (batch_write_t*) arg;
    w->ok            = bra_io_file_write(w->dst, w->buf, (size_t) w->n);
    return NULL;
}

static void batch_write_start(batch_write_t* w, bra_io_file_t* dst, const uint8_t* buf, uint64_t n)
{
    w->dst = dst, w->buf = buf, w->n = n, w->ok = false;
    w->running = pthread_create(&w->th, NULL, batch_write_main, w) == 0;
    if (!w->running)
        w->ok = bra_io_file_write(dst, buf, (size_t) n);
}

static bool batch_write_join(batch_write_t* w)
{
    if (w->running)
        pthread_join(w->th, NULL);
    w->running = false;
    return w->ok;
}

/* Pinned decode buffers (kept across files): two record batches and two decoded batches. */
static uint8_t* g_dec_stream[2];
static uint8_t* g_dec_out[2];
static uint64_t g_dec_scap, g_dec_ocap;

static void front_dec_release(void)
{
    for (int q = 0; q < 2; ++q)
    {
        bra_gpu_host_free(g_front_ctx, g_dec_stream[q]);
        bra_gpu_host_free(g_front_ctx, g_dec_out[q]);
        g_dec_stream[q] = g_dec_out[q] = NULL;
    }
    g_dec_scap = g_dec_ocap = 0;
}

static bool front_dec_bufs(bra_gpu_ctx_t* ctx, uint64_t scap, uint64_t ocap)
{
    if (scap > g_dec_scap || ocap > g_dec_ocap)
    {
        front_dec_release();
        bool ok = true;
        for (int q = 0; q < 2; ++q)
        {
            g_dec_stream[q] = (uint8_t*) bra_gpu_host_alloc(ctx, scap);
            g_dec_out[q]    = (uint8_t*) bra_gpu_host_alloc(ctx, ocap);
            ok              = ok && g_dec_stream[q] != NULL && g_dec_out[q] != NULL;
        }
        if (!ok)
        {
            front_dec_release();
            return false;
        }
        g_dec_scap = scap, g_dec_ocap = ocap;
    }
    return true;
}

bool bra_io_file_chunks_decompress_file(bra_io_file_t* dst, bra_io_file_t* src, const uint64_t data_size, bra_meta_entry_t* me, const bool decode)
{
    assert(src != NULL && me != NULL);
    const int      tm      = front_timing();
    const double   t0      = tm ? now_ms() : 0;
    double         t_parse = 0, t_dev = 0, t_wait = 0, tt = 0;
    bra_gpu_ctx_t* ctx     = decode ? front_ctx() : NULL;
    bool           ok      = !(dst != NULL && (dst->f == NULL || dst->fn == NULL)) && (!decode || ctx != NULL);
    // a batch holds whole records: up to BATCH_CHUNKS of them, at most that many chunk sizes of
    // decoded output (the headers bound every chunk by BRA_MAX_CHUNK_SIZE)
    const uint64_t rec_max = sizeof(bra_huffman_t) + BRA_BWT_INDEX_BYTES + CHUNK_SIZE;
    const uint64_t scap    = (uint64_t) BATCH_CHUNKS * rec_max;
    const uint64_t ocap    = (uint64_t) (BATCH_CHUNKS < 2 ? 2 : BATCH_CHUNKS) * CHUNK_SIZE;
    uint8_t*       lst     = NULL;  // listing (decode == false): a plain record buffer
    if (ok && decode)
        ok = front_dec_bufs(ctx, scap, ocap);
    else if (ok)
        ok = (lst = (uint8_t*) malloc(scap)) != NULL;
    const double  t_ctx = tm ? now_ms() - t0 : 0;
    uint64_t      orig  = 0;
    batch_write_t wr;
    memset(&wr, 0, sizeof wr);
    wr.ok = true;
    for (uint64_t done = 0, k = 0; ok && done < data_size; ++k)
    {
        uint8_t* stream  = decode ? g_dec_stream[k % 2] : lst;
        uint8_t* decoded = decode ? g_dec_out[k % 2] : NULL;
        // read up to BATCH_CHUNKS records (header, check, payload) into the stream buffer; a bad
        // header or a failed read ends the batch after the good records before it
        uint64_t fill = 0;
        uint32_t recs = 0;
        bool     bad  = false;
        tt            = tm ? now_ms() : 0;
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
        t_parse += tm ? now_ms() - tt : 0;
        if (decode && recs > 0)
        {
            // the reference writes every chunk before a bad record: decode the good ones first.
            // decoded[k % 2] was last written out by batch k - 2's writer, joined below (batch
            // k - 1's) or at the previous iteration
            tt            = tm ? now_ms() : 0;
            uint64_t  osz = 0;
            uint32_t  crc = me->crc32;
            const int rc  = bad ? -1 : bra_gpu_decompress_chunks_host(ctx, stream, fill, (uint32_t) CHUNK_SIZE, decoded, ocap, &osz, me->crc32, &crc, 0);
            t_dev += tm ? now_ms() - tt : 0;
            tt = tm ? now_ms() : 0;
            ok = batch_write_join(&wr);  // batch k - 1 is on disk: decoded[(k + 1) % 2] is free again
            t_wait += tm ? now_ms() - tt : 0;
            if (ok && rc == 0)
            {
                me->crc32 = crc;
                orig += osz;
                if (dst != NULL && osz > 0)
                    batch_write_start(&wr, dst, decoded, osz);
            }
            else if (ok)
                ok = decode_records_serial(dst, src->fn, stream, recs, me, &orig, g_dec_out[(k + 1) % 2]) && !bad;
        }
        ok = ok && !bad;
        done += fill;
    }
    tt = tm ? now_ms() : 0;
    if (!batch_write_join(&wr))
        ok = false;
    t_wait += tm ? now_ms() - tt : 0;
    if (ok && orig <= data_size)
    {
        bra_log_error("corrupted file entry: %s", me->name);
        ok = false;
    }
    if (ok)
        me->_compression_ratio = (float) ((double) data_size / (double) orig);
    free(lst);
    if (tm && decode)
        fprintf(stderr, "front: decompress %" PRIu64 " bytes into %" PRIu64 " in %.1f ms: ctx+buffers %.1f, record reads %.1f, device %.1f, write waits %.1f\n",
                data_size, orig, now_ms() - t0, t_ctx, t_parse, t_dev, t_wait);
    if (!ok)
    {
        if (dst != NULL && dst->f != NULL)
            bra_io_file_close(dst);
        bra_io_file_close(src);
    }
    return ok;
}
