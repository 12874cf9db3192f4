/*
 * ref_chunks.c -- TEST INFRASTRUCTURE ONLY.  A driver compiled together with the reference's
 * lib_bra sources (oracle/Makefile, target `ref`) into oracle/_ref/libbralib.so.  It runs the
 * reference's own chunk loop, bra_io_file_chunks_compress_file (src/io/lib_bra_io_file_chunks.c:
 * 169-312), on one file, so the tests can compare the GPU batched chunk loop (row f1) and the
 * device CRC32C (row f2) with the exact bytes and CRC the reference produces.
 */
#include <lib_bra.h>
#include <lib_bra_defs.h>
#include <io/lib_bra_io_file.h>
#include <io/lib_bra_io_file_chunks.h>

#include <stdint.h>
#include <string.h>

/* Compress src_fn (size bytes) with the reference chunk loop into dst_fn.  Returns 1 on success;
 * the meta entry's CRC before and after, and its attributes after (compressed or stored). */
int ref_compress_file(const char* src_fn, const char* dst_fn, uint64_t size, uint32_t* crc_before, uint32_t* crc_after, uint32_t* attr_after)
{
    if (!bra_init())
        return 0;
    bra_io_file_t src, dst;
    memset(&src, 0, sizeof src);
    memset(&dst, 0, sizeof dst);
    int ok = 0;
    if (bra_io_file_open(&src, src_fn, "rb") && bra_io_file_open(&dst, dst_fn, "wb"))
    {
        bra_meta_entry_t me;
        memset(&me, 0, sizeof me);
        if (bra_meta_entry_init(&me, BRA_ATTR_SET_COMP(BRA_ATTR_TYPE_FILE, BRA_ATTR_COMP_COMPRESSED), "f", 1) && bra_meta_entry_file_set(&me, size))
        {
            *crc_before = me.crc32;
            ok          = bra_io_file_chunks_compress_file(&dst, &src, size, &me) ? 1 : 0;
            *crc_after  = me.crc32;
            *attr_after = me.attributes;
        }
        bra_meta_entry_free(&me);
    }
    bra_io_file_close(&src);
    bra_io_file_close(&dst);
    bra_quit();
    return ok;
}

/* Decode `size` bytes of chunk records (what ref_compress_file writes after the 8-byte data size)
 * with the reference's bra_io_file_chunks_decompress_file (lib_bra_io_file_chunks.c:314-441) into
 * dst_fn.  Returns 1 on success, 0 when the reference rejects the stream (e.g. a chunk header whose
 * encoded_size exceeds BRA_MAX_CHUNK_SIZE, :36-40); *crc_after = the entry CRC it accumulated. */
int ref_decompress_file(const char* src_fn, const char* dst_fn, uint64_t size, uint32_t* crc_after)
{
    if (!bra_init())
        return 0;
    bra_io_file_t src, dst;
    memset(&src, 0, sizeof src);
    memset(&dst, 0, sizeof dst);
    int ok = 0;
    if (bra_io_file_open(&src, src_fn, "rb") && bra_io_file_open(&dst, dst_fn, "wb"))
    {
        bra_meta_entry_t me;
        memset(&me, 0, sizeof me);
        if (bra_meta_entry_init(&me, BRA_ATTR_SET_COMP(BRA_ATTR_TYPE_FILE, BRA_ATTR_COMP_COMPRESSED), "f", 1) && bra_meta_entry_file_set(&me, size))
        {
            ok         = bra_io_file_chunks_decompress_file(&dst, &src, size, &me, true) ? 1 : 0;
            *crc_after = me.crc32;
        }
        bra_meta_entry_free(&me);
    }
    bra_io_file_close(&src);
    bra_io_file_close(&dst);
    bra_quit();
    return ok;
}
