/*
 * bra_hip.h -- C-ABI of the MI355X (gfx950) block codec: a drop-in for the reference's lib_bra
 * encoder/decoder entry points plus a batched device-resident extension.
 *
 * Part 1 re-exports the 14 functions of the reference's src/encoders headers with identical
 * signatures, memory ownership and error behaviour, so that lib_bra's chunk loop
 * (src/io/lib_bra_io_file_chunks.c:217-262, :362-393) and therefore bra / unbra / bra.sfx link
 * against libbra_hip.so unchanged.  Every call runs on the GPU; there is no
 * CPU code path.  A process-wide device context is created lazily on first use (the reference
 * tests call the encoders without bra_init(), test/test_bra_encoders.cpp); calls are serialised.
 *
 * Part 2 is the batch API the throughput path uses: many independent blocks, all buffers already
 * in HBM, one call.
 */
#pragma once

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- ABI types (same layout as src/lib_bra_types.h:11, :51-56, :63-68; src/encoders/bra_huffman.h:13-17) ---- */
#ifndef BRA_HIP_NO_TYPES
typedef uint32_t bra_bwt_index_t;

#pragma pack(push, 1)
typedef struct bra_huffman_t
{
    uint8_t  lengths[256]; /* canonical code length per symbol, 0 = absent */
    uint32_t orig_size;    /* Huffman input (= RLE output) size */
    uint32_t encoded_size; /* payload bytes */
} bra_huffman_t;
#pragma pack(pop)

typedef struct bra_huffman_chunk_t
{
    bra_huffman_t meta;
    uint8_t*      data;
} bra_huffman_chunk_t;

typedef struct bra_io_chunk_header_t
{
    bra_bwt_index_t primary_index;
    bra_huffman_t   huffman;
} bra_io_chunk_header_t;
#endif

/* ---- Part 1: reference encoder ABI ---------------------------------------------------------- */
/* replaces src/encoders/bra_bwt.h:42  (bra_bwt.c:57-71)   */
uint8_t* bra_bwt_encode(const uint8_t* buf, const bra_bwt_index_t buf_size, bra_bwt_index_t* primary_index);
/* replaces src/encoders/bra_bwt.h:63  (bra_bwt.c:73-108)  */
bool bra_bwt_encode2(const uint8_t* buf, const bra_bwt_index_t buf_size, bra_bwt_index_t* primary_index, uint8_t* out_buf);
/* replaces src/encoders/bra_bwt.h:93  (bra_bwt.c:110-131) */
uint8_t* bra_bwt_decode(const uint8_t* buf, const bra_bwt_index_t buf_size, const bra_bwt_index_t primary_index);
/* replaces src/encoders/bra_bwt.h:124 (bra_bwt.c:133-168) */
void bra_bwt_decode2(const uint8_t* buf, const bra_bwt_index_t buf_size, const bra_bwt_index_t primary_index, bra_bwt_index_t* transform,
                     uint8_t* out_buf);
/* replaces src/encoders/bra_mtf.h:29  (bra_mtf.c:48-65)   */
uint8_t* bra_mtf_encode(const uint8_t* buf, const size_t buf_size);
/* replaces src/encoders/bra_mtf.h:51  (bra_mtf.c:67-82)   */
bool bra_mtf_encode2(const uint8_t* buf, const size_t buf_size, uint8_t* out_buf);
/* replaces src/encoders/bra_mtf.h:70  (bra_mtf.c:84-96)   */
uint8_t* bra_mtf_decode(const uint8_t* buf, const size_t buf_size);
/* replaces src/encoders/bra_mtf.h:83  (bra_mtf.c:98-115)  */
void bra_mtf_decode2(const uint8_t* buf, const size_t buf_size, uint8_t* out_buf);
/* replaces src/encoders/bra_rle.h:24  (bra_rle.c:60-120)  -- *out_buf is malloc() memory */
bool bra_rle_encode(const uint8_t* buf, const size_t buf_size, uint8_t** out_buf, size_t* out_buf_size);
/* replaces src/encoders/bra_rle.h:33  (bra_rle.c:122-160) -- 0 on a malformed stream */
size_t bra_rle_decode_compute_size(const uint8_t* buf, const size_t buf_size);
/* replaces src/encoders/bra_rle.h:47  (bra_rle.c:162-224) -- *out_buf is malloc() memory */
bool bra_rle_decode(const uint8_t* buf, const size_t buf_size, uint8_t** out_buf, size_t* out_buf_size);
/* replaces src/encoders/bra_huffman.h:25 (bra_huffman.c:352-432) -- NULL when buf_size == 0 */
bra_huffman_chunk_t* bra_huffman_encode(const uint8_t* buf, const uint32_t buf_size);
/* replaces src/encoders/bra_huffman.h:35 (bra_huffman.c:434-498) -- malloc() memory or NULL */
uint8_t* bra_huffman_decode(const bra_huffman_t* meta, const uint8_t* data, uint32_t* out_size);
/* replaces src/encoders/bra_huffman.h:42 (bra_huffman.c:500-512) */
void bra_huffman_chunk_free(bra_huffman_chunk_t* chunk);

/* ---- Part 2: batched, device-resident block codec -------------------------------------------- */
typedef struct bra_gpu_ctx_s bra_gpu_ctx_t;

/* A context owns device scratch (grown on demand) and a HIP stream on `device`.  NULL on error. */
bra_gpu_ctx_t* bra_gpu_ctx_create(int device);
void           bra_gpu_ctx_destroy(bra_gpu_ctx_t* ctx);

/* Number of blocks `total` bytes split into blocks of `block_size` bytes (last block ragged). */
uint32_t bra_gpu_num_blocks(uint64_t total, uint32_t block_size);

/* Payload capacity for bra_gpu_encode_blocks of this geometry when no code is longer than 32 bits
 * (always true below ~3.5 M symbols per block); a call that needs more fails with -2 and leaves the
 * required size in d_payload_off[nblocks]. */
uint64_t bra_gpu_payload_bound(uint64_t total, uint32_t block_size);

/*
 * Encode every block of d_in[0, total) (device memory) with BWT -> MTF -> RLE -> Huffman, exactly
 * as bra_io_file_chunks_compress_file does per chunk (lib_bra_io_file_chunks.c:217-245).
 *   d_headers[b]       pi + bra_huffman_t of block b (the 268-byte in-memory chunk header)
 *   d_payload_off[b]   byte offset of block b's Huffman payload in d_payload (nblocks+1 entries;
 *                      the last one is the total payload size)
 *   d_payload          payloads back to back, capacity payload_cap bytes
 * block_size must be in [1, 2^24); the stream may be NULL (context stream).
 * Returns 0 on success, < 0 on error (logged through bra_log_error when lib_bra is linked).
 */
int bra_gpu_encode_blocks(bra_gpu_ctx_t* ctx, const uint8_t* d_in, uint64_t total, uint32_t block_size, bra_io_chunk_header_t* d_headers,
                          uint64_t* d_payload_off, uint8_t* d_payload, uint64_t payload_cap, void* stream);

/*
 * Inverse of bra_gpu_encode_blocks: reconstruct d_out[0, total) from the headers and payloads.
 * Fails (< 0) on any block the reference decoder would reject or whose size differs from the
 * geometry (total, block_size).
 */
int bra_gpu_decode_blocks(bra_gpu_ctx_t* ctx, const bra_io_chunk_header_t* d_headers, const uint64_t* d_payload_off,
                          const uint8_t* d_payload, uint64_t total, uint32_t block_size, uint8_t* d_out, void* stream);

/*
 * Device pointers to the intermediate stage outputs of the last bra_gpu_encode_blocks call (for
 * parity tests): 0 = BWT last column (total bytes), 1 = MTF (total bytes), 2 = RLE output (block b
 * at byte offset rle_base[b]), 3 = rle_base (uint64_t[nblocks]), 4 = RLE sizes (uint32_t[nblocks]).
 */
const void* bra_gpu_stage_ptr(bra_gpu_ctx_t* ctx, int stage);

/*
 * Kernel timing with HIP events on the launching stream (used by bench.py): `mask` selects the
 * timing slots (bit i = slot i; 0 = off).  bra_gpu_prof_read waits for the recorded events and
 * returns the number of slots; for a valid `slot` it reports the slot's name, the summed device
 * time in ms, the number of launches timed since the last reset and their algorithmic HBM bytes
 * (the bytes the algorithm must move, DESIGN.md "Roofline"), so bytes / time is achieved GB/s.
 */
void bra_gpu_prof_enable(bra_gpu_ctx_t* ctx, uint64_t mask);
void bra_gpu_prof_reset(bra_gpu_ctx_t* ctx);
int  bra_gpu_prof_read(bra_gpu_ctx_t* ctx, int slot, const char** name, double* total_ms, uint32_t* launches, double* bytes);

/* Library identification for the loader tests. */
const char* bra_gpu_version(void);

#ifdef __cplusplus
}
#endif
