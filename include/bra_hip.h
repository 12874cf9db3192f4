/*
 * bra_hip.h -- C-ABI of the MI355X (gfx950) block codec: a drop-in for the reference's lib_bra
 * encoder/decoder entry points plus a batched device-resident extension.
 *
 * Part 1 re-exports the 14 functions of the reference's src/encoders headers with identical
 * signatures, memory ownership and error behaviour, so that lib_bra's chunk loop
 * (src/io/lib_bra_io_file_chunks.c:217-262, :362-393) and therefore bra / unbra / bra.sfx link
 * against libbra_hip.so unchanged.  Every call runs on the GPU; there is no
 * CPU code path.  No bra_init() is needed (the reference tests call the encoders without it,
 * test/test_bra_encoders.cpp): a call leases a device context from a per-device pool for the
 * calling thread's current HIP device (created on first use), so concurrent callers run on
 * separate contexts and the functions are re-entrant as the reference's are.
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
/* replaces src/encoders/bra_bwt.h:63  (bra_bwt.c:73-108); any length >= 1 (blocks of 2^24 bytes or
   more take the prefix-doubling path of csrc/bwt_large.hip) */
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

/* A context owns device scratch (grown on demand) and a HIP stream on `device` (-1: the calling
 * thread's current device).  NULL on error. */
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

/* ---- Part 3: the .BRa chunk stream on the device --------------------- */
/* Streams: a NULL stream means the context's stream and the call has completed when it returns;
 * with an explicit stream the device results are ordered on that stream. */

/*
 * CRC32C of d_data[0, len) (device memory) chained from prev, i.e. bra_crc32c(data, len, prev)
 * (replaces src/utils/lib_bra_crc32c.h bra_crc32c, lib_bra_crc32c.c:102-117 / :133-179 for
 * device-resident data).  The result is written to *d_crc (device memory) on the stream.
 */
int bra_gpu_crc32c(bra_gpu_ctx_t* ctx, const void* d_data, uint64_t len, uint32_t prev, uint32_t* d_crc, void* stream);

/*
 * CRC32C of the chunk stream hdr[0] || chunk 0 || hdr[1] || chunk 1 || ... chained from prev, where
 * hdr[b] is the 268-byte in-memory header d_headers[b] and chunk b is d_data[b*block_size, ...)
 * (last one ragged).  prev = 0 (BRA_CRC32C_INIT) gives the `crc32` of the reference compress loop
 * (lib_bra_io_file_chunks.c:214,248-249); prev = me->crc32 over decoded chunks gives the decode
 * loop's update (:396-397).  Result in *d_crc (device memory).
 */
int bra_gpu_chunks_crc32c(bra_gpu_ctx_t* ctx, const uint8_t* d_data, uint64_t total, uint32_t block_size,
                          const bra_io_chunk_header_t* d_headers, uint32_t prev, uint32_t* d_crc, void* stream);

/* Host: bra_crc32c_combine (lib_bra_crc32c.c:181-231) with a 64-bit length; used to merge the
 * per-rank chunk-stream CRCs of a sharded encode in block order. */
uint32_t bra_gpu_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* Host: me->crc32 after a compressed file (lib_bra_io_file_chunks.c:291-292) from the meta entry's
 * CRC so far, the chunk stream size (tmpfile size), its CRC and the input size.  The combine
 * length is truncated to 32 bits exactly as in the reference. */
uint32_t bra_gpu_entry_crc32c(uint32_t me_crc, uint64_t chunks_size, uint32_t chunks_crc, uint64_t data_size, uint32_t block_size);

/* Output capacity for bra_gpu_compress_chunks: payload bound + 267 bytes per chunk. */
uint64_t bra_gpu_chunks_bound(uint64_t total, uint32_t block_size);
/* Output capacity for bra_gpu_compress_chunks_collect of one batch of total bytes: the chunk records
 * the pipelined API can return (RLE-capacity payloads + 267 bytes per chunk), about 1.01x total. */
uint64_t bra_gpu_pipe_records_bound(uint64_t total, uint32_t block_size);

/*
 * Write the .BRa chunk records of nblocks encoded blocks (bra_gpu_encode_blocks output) back to
 * back into d_out: 3 low bytes of pi + the packed 264-byte bra_huffman_t + payload
 * (bra_io_file_chunks_write_header, lib_bra_io_file_chunks.c:76-95, then :260).  *out_size =
 * payload_off[nblocks] + 267 * nblocks; -2 when that exceeds out_cap.
 */
int bra_gpu_frame_chunks(bra_gpu_ctx_t* ctx, const bra_io_chunk_header_t* d_headers, const uint64_t* d_payload_off, const uint8_t* d_payload,
                         uint32_t nblocks, uint8_t* d_out, uint64_t out_cap, uint64_t* out_size, void* stream);

/*
 * Parse a chunk stream d_stream[0, stream_size) (the read loop of bra_io_file_chunks_decompress_file,
 * lib_bra_io_file_chunks.c:340-420): headers to d_headers, payload b at d_stream + d_payload_off[b].
 * Fails (< 0) on a truncated stream, more than max_chunks records, or a header that
 * bra_io_file_chunks_header_validate (:31-49) rejects.  *n_chunks = records found.
 */
int bra_gpu_unframe_chunks(bra_gpu_ctx_t* ctx, const uint8_t* d_stream, uint64_t stream_size, uint32_t max_chunks,
                           bra_io_chunk_header_t* d_headers, uint64_t* d_payload_off, uint32_t* n_chunks, void* stream);

/*
 * The compress chunk loop (bra_io_file_chunks_compress_file, lib_bra_io_file_chunks.c:199-278) over
 * device data: every block_size chunk of d_in[0, data_size) encoded, framed into d_out (the exact
 * bytes the reference writes to its tmpfile, *out_size of them) and the loop's running CRC32C in
 * *chunks_crc (host).  block_size = 262144 (BRA_MAX_CHUNK_SIZE) reproduces the reference format.
 * Returns 1 when the chunk stream is smaller than the input, 0 when it is not (the reference then
 * stores the file: BRA_ATTR_COMP_STORED, :274-278), -2 when out_cap is too small (*out_size holds
 * the need), other < 0 on error.  Pair with bra_gpu_entry_crc32c for me->crc32.
 */
int bra_gpu_compress_chunks(bra_gpu_ctx_t* ctx, const uint8_t* d_in, uint64_t data_size, uint32_t block_size, uint8_t* d_out,
                            uint64_t out_cap, uint64_t* out_size, uint32_t* chunks_crc, void* stream);

/*
 * The decode loop (bra_io_file_chunks_decompress_file, lib_bra_io_file_chunks.c:340-427) over a
 * device-resident chunk stream: the decoded bytes back to back in d_out (*out_size of them, at
 * most out_cap; -2 if larger) and, when crc_out is non-NULL, me->crc32 updated from prev_crc as the
 * reference does (:396-397).  Every reference rejection is an error here too (invalid header,
 * Huffman / RLE failure, pi >= chunk size, decoded size not above the stream size).  block_size
 * bounds every chunk's decoded size.
 */
int bra_gpu_decompress_chunks(bra_gpu_ctx_t* ctx, const uint8_t* d_stream, uint64_t stream_size, uint32_t block_size, uint8_t* d_out,
                              uint64_t out_cap, uint64_t* out_size, uint32_t prev_crc, uint32_t* crc_out, void* stream);

/*
 * Host-buffer forms of the two chunk loops, for a C front end that replaces lib_bra's
 * src/io/lib_bra_io_file_chunks.c (frontend/bra_io_file_chunks_gpu.c): the input
 * is staged into the context's device buffers, the device loop runs, the result is copied back to
 * h_out; the call has completed when it returns.  Return codes as the device forms.  For the
 * decode, whole_entry != 0 applies the reference's end-of-entry check (decoded size above the
 * stream size, lib_bra_io_file_chunks.c:423-427); a caller decoding one entry in several batches
 * passes 0 and checks the total itself.
 */
int bra_gpu_compress_chunks_host(bra_gpu_ctx_t* ctx, const uint8_t* h_in, uint64_t data_size, uint32_t block_size, uint8_t* h_out,
                                 uint64_t out_cap, uint64_t* out_size, uint32_t* chunks_crc);
int bra_gpu_decompress_chunks_host(bra_gpu_ctx_t* ctx, const uint8_t* h_stream, uint64_t stream_size, uint32_t block_size, uint8_t* h_out,
                                   uint64_t out_cap, uint64_t* out_size, uint32_t prev_crc, uint32_t* crc_out, int whole_entry);

/*
 * The same compression with two batches in flight (the front end's overlapped batch loop, replacing
 * the reference's per-chunk loop lib_bra_io_file_chunks.c:199-266).  bra_gpu_compress_chunks_stage
 * queues the copy of h_in into slot 0 or 1 on the context's input-copy stream, behind the device's
 * use of the slot's previous batch; bra_gpu_compress_chunks_submit queues the slot's encode, framing
 * and chunk-stream CRC behind that copy (it makes the copy itself when the slot has none staged; a
 * staged slot must be submitted with the same h_in and data_size) and returns once the batch's BWT
 * jobs are done, with the rest of the batch still queued; h_in may be refilled from then on.
 * bra_gpu_compress_chunks_collect waits for the slot's batch, copies its chunk records into h_out on
 * the output-copy stream and returns what bra_gpu_compress_chunks_host returns (1 smaller than the
 * input, 0 not smaller, -2 out_cap too small: *out_size = the bytes needed and the batch stays in
 * the slot, so a second collect with a larger buffer returns it; -1 error); a slot is
 * collected before it is submitted again.  Collect with h_out NULL drains the slot: it waits for the
 * submitted batch and drops it, and drops a staged copy.  Other calls on the context may be made
 * while a batch is in flight: a call on a caller-supplied stream waits on the device for the
 * in-flight batches, and the next submit for the last such call (they share the context's work
 * buffers).  The overlapped order: stage(k + 1) before submit(k)
 * (batch k + 1's input arrives while batch k's kernels run), then collect(k - 1) (its records return
 * under batch k's kernels).  Host buffers from bra_gpu_host_alloc (pinned) make the copies
 * asynchronous; bra_gpu_host_free releases them.
 */
void* bra_gpu_host_alloc(bra_gpu_ctx_t* ctx, uint64_t bytes);
void  bra_gpu_host_free(bra_gpu_ctx_t* ctx, void* p);
int   bra_gpu_compress_chunks_stage(bra_gpu_ctx_t* ctx, int slot, const uint8_t* h_in, uint64_t data_size);
int   bra_gpu_compress_chunks_submit(bra_gpu_ctx_t* ctx, int slot, const uint8_t* h_in, uint64_t data_size, uint32_t block_size);
int   bra_gpu_compress_chunks_collect(bra_gpu_ctx_t* ctx, int slot, uint8_t* h_out, uint64_t out_cap, uint64_t* out_size, uint32_t* chunks_crc);

/* ---- Part 4: blocks sharded over several GPUs (SURVEY 8.1 row e) ----------------------------- */

/*
 * One shard's share of bra_gpu_chunks_crc32c over a stream whose chunks are spread over devices:
 * this device holds global chunks first_chunk, first_chunk + chunk_stride, ... back to back in
 * d_data[0, total) with their headers in d_headers (every chunk block_size bytes except the global
 * last, which must then be this shard's last).  The XOR of all shards' *d_crc words is the CRC32C of
 * the whole global_total-byte chunk stream chained from prev, when exactly one shard passes
 * with_init != 0.  Round-robin sharding over G ranks: first_chunk = rank, chunk_stride = G.
 */
int bra_gpu_chunks_crc32c_shard(bra_gpu_ctx_t* ctx, const uint8_t* d_data, uint64_t total, uint32_t block_size,
                                const bra_io_chunk_header_t* d_headers, uint64_t first_chunk, uint64_t chunk_stride, uint64_t global_total,
                                uint32_t prev, int with_init, uint32_t* d_crc, void* stream);

/*
 * Assemble the bra_gpu_encode_blocks outputs of nparts (<= 16) shards, all resident on this
 * context's device, into global block order: headers, payload offsets (N + 1 entries, N = sum of
 * nblocks[]) and payloads back to back.  round_robin != 0: global block g is shard g % nparts's
 * block g / nparts; otherwise shard p holds the next nblocks[p] blocks.  With stream == NULL it
 * completes before returning and returns 0, -2 when the payloads need more than payload_cap bytes
 * (d_payload_off_out[N] then holds the payload size needed), -1 on error.  With a stream it returns 0
 * once queued (-1 on an argument error) and an overflow shows on the device as
 * d_payload_off_out[N] == UINT64_MAX (the blocks past payload_cap are then not copied; the size
 * needed is the sum of the parts' d_payload_off[p][nblocks[p]]).
 */
int bra_gpu_assemble_shards(bra_gpu_ctx_t* ctx, uint32_t nparts, const bra_io_chunk_header_t* const* d_headers,
                            const uint64_t* const* d_payload_off, const uint8_t* const* d_payload, const uint32_t* nblocks, int round_robin,
                            bra_io_chunk_header_t* d_headers_out, uint64_t* d_payload_off_out, uint8_t* d_payload_out, uint64_t payload_cap,
                            void* stream);

/*
 * Device pointers to the intermediate stage outputs of the last bra_gpu_encode_blocks call (for
 * parity tests): 0 = BWT last column (total bytes), 1 = MTF (total bytes), 2 = RLE output (block b
 * at byte offset rle_base[b]), 3 = rle_base (uint64_t[nblocks]), 4 = RLE sizes (uint32_t[nblocks]),
 * 5 = BWT suffix-array slots (uint32_t per input byte, block-local rotation indices at the block
 * offsets).
 */
const void* bra_gpu_stage_ptr(bra_gpu_ctx_t* ctx, int stage);

/*
 * Diagnostics of the BWT job kernels (no reference equivalent; tests/test_gpu_jobs.py).
 * bra_gpu_debug_rerun_jobs re-runs the job phase of the last batch encode `reps` times on its
 * unchanged job lists -- with every job's input payloads put in another order first when
 * shuffle_seed != 0 -- and checks each run (no slot covered by two jobs, every job's output
 * rotations = its input rotations); returns the failing jobs summed over the runs, -1 on an error
 * or when there is nothing to re-run: only right after a batch encode on the context (no decode or
 * fallback since), with that encode's input buffer still allocated and unchanged.
 * bra_gpu_sortnet_selftest: waves must be 1, 2 or 4 and groups >= 1 (else -1).
 * bra_gpu_sortnet_selftest sorts groups x iters random key sets (or the 256 * waves given keys,
 * slot order, padding all ones) with the job sort of `waves` waves and returns the failing sorts.
 */
int bra_gpu_debug_rerun_jobs(bra_gpu_ctx_t* ctx, int reps, unsigned shuffle_seed);
int bra_gpu_sortnet_selftest(int waves, unsigned groups, unsigned iters, unsigned seed, const unsigned long long* keys);

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

/*
 * Device self-test of the wave / workgroup scan primitives the kernels are built from (lane
 * exchanges through DPP, readlane and ds_bpermute): 0 = all match a serial restatement, > 0 =
 * number of mismatches, < 0 = HIP error.  Diagnostics only; no codec state is touched.
 */
int bra_gpu_selftest(void);

#ifdef __cplusplus
}
#endif
