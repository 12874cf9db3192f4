// crc.h -- CRC32C of the .BRa chunk stream and chunk framing on the device.
#pragma once

#include "bra_hip_common.h"

namespace bra {

constexpr uint32_t CHUNK_HDR_MEM  = 268;  // sizeof(bra_io_chunk_header_t) (lib_bra_types.h:63-68)
constexpr uint32_t CHUNK_HDR_DISK = 267;  // BRA_IO_CHUNK_HEADER_SIZE (lib_bra_defs.h:99)
constexpr uint32_t BRA_MAX_CHUNK  = 256 * 1024;  // BRA_MAX_CHUNK_SIZE (lib_bra_defs.h:93)

// Host GF(2) arithmetic for the reflected CRC32C polynomial (same algebra as the device code).
uint32_t crc_mulmod(uint32_t a, uint32_t b);           // a * b mod P
uint32_t crc_x8n(uint64_t nbytes);                     // x^(8 * nbytes) mod P
uint32_t crc32c_host(const void* data, uint64_t len, uint32_t prev);  // == bra_crc32c
uint32_t crc32c_combine_host(uint32_t a, uint32_t b, uint64_t len_b);  // == bra_crc32c_combine

// CRC32C, chained from `prev` like bra_crc32c(data, len, prev), of the virtual stream
//     hdr[0] || data[chunk 0] || hdr[1] || data[chunk 1] || ...
// where chunk b is data[b * chunk_size, min(total, (b + 1) * chunk_size)) and hdr[b] the 268-byte
// in-memory chunk header at d_hdr + 268 * b.  With d_hdr == nullptr the stream is data alone
// (plain CRC32C of a device buffer).  The result lands in *d_crc (device memory) on stream s.
bool crc_stream_device(const uint8_t* d_data, uint64_t total, uint32_t chunk_size, const uint8_t* d_hdr, uint32_t prev, uint32_t* d_crc,
                       hipStream_t s);

// The same CRC for one shard of a stream whose chunks are spread over several devices: this
// device's data holds global chunks g0, g0 + gstride, g0 + 2*gstride, ... back to back (chunks of
// chunk_size bytes; only the global last chunk, which must then be this shard's last, is ragged)
// and d_hdr their headers.  *d_crc receives the shard's share of the CRC of the whole
// global_total-byte stream: XOR over the shards gives bra_crc32c of the stream chained from `prev`,
// when exactly one shard passes with_init = true.  Round-robin sharding: g0 = rank, gstride = world.
bool crc_stream_shard_device(const uint8_t* d_data, uint64_t total, uint32_t chunk_size, const uint8_t* d_hdr, uint64_t g0, uint64_t gstride,
                             uint64_t global_total, uint32_t prev, bool with_init, uint32_t* d_crc, hipStream_t s);

// Write the .BRa chunk records (3-byte pi + 264-byte bra_huffman_t + payload, lib_bra_io_file_chunks.c:
// 76-95,260) of nb chunks back to back into d_out.  Record b starts at payload_off[b] + 267 * b.
bool frame_chunks_device(const uint8_t* d_hdr, const uint64_t* d_payload_off, const uint8_t* d_payload, uint32_t nb, uint8_t* d_out,
                         hipStream_t s);

// Inverse of the framing: walk the records of d_stream[0, size) (lib_bra_io_file_chunks.c:340-420
// loop), validate each header like bra_io_file_chunks_header_validate (:31-49, with max_chunk as
// BRA_MAX_CHUNK_SIZE) and emit the 268-byte headers plus each payload's offset in d_stream.
// d_status receives {number of records, error flag}; cap is the capacity of d_hdr / d_payload_off.
bool unframe_chunks_device(const uint8_t* d_stream, uint64_t size, uint32_t cap, uint32_t max_chunk, uint8_t* d_hdr, uint64_t* d_payload_off,
                           uint32_t* d_status, hipStream_t s);

// Encoder output of up to MAX_SHARDS devices (headers, payload offsets, payloads; device memory of
// the assembling device).  Global block g is part g % n's local block g / n with round_robin, else
// part p holds the contiguous global blocks [first[p], first[p + 1]).
constexpr uint32_t MAX_SHARDS = 16;
struct ShardParts
{
    const uint8_t*  hdr[MAX_SHARDS];
    const uint64_t* off[MAX_SHARDS];
    const uint8_t*  pay[MAX_SHARDS];
    uint32_t        first[MAX_SHARDS + 1];
    uint32_t        n;
    uint32_t        round_robin;
};

// Headers, payload offsets (nb + 1 entries) and payloads of all nb global blocks in global order;
// *d_err != 0 when the payloads need more than cap bytes (d_off_out[nb] is then UINT64_MAX); *d_need
// receives the payload size the assembly needs either way.
bool assemble_shards_device(const ShardParts& parts, uint32_t nb, uint8_t* d_hdr_out, uint64_t* d_off_out, uint8_t* d_pay_out, uint64_t cap,
                            uint32_t* d_err, uint64_t* d_need, hipStream_t s);

}  // namespace bra
