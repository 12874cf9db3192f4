/*
 * oracle/bra_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference encoder
 * chain, used as the parity checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  Never linked into the product library (br-archive_amd/).
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field layout as bra_huffman_t (src/lib_bra_types.h:51-56), packed. */
#pragma pack(push, 1)
typedef struct orc_huffman_meta_t
{
    uint8_t  lengths[256];
    uint32_t orig_size;
    uint32_t encoded_size;
} orc_huffman_meta_t;
#pragma pack(pop)

int    orc_bwt_encode(const uint8_t* in, uint32_t n, uint32_t* primary_index, uint8_t* out, uint32_t* sa_out);
int    orc_bwt_decode(const uint8_t* in, uint32_t n, uint32_t primary_index, uint8_t* out);
int    orc_mtf_encode(const uint8_t* in, size_t n, uint8_t* out);
int    orc_mtf_decode(const uint8_t* in, size_t n, uint8_t* out);
size_t orc_rle_encode(const uint8_t* in, size_t n, uint8_t* out); /* out may be NULL: size only */
size_t orc_rle_decode_size(const uint8_t* in, size_t n);
size_t orc_rle_decode(const uint8_t* in, size_t n, uint8_t* out);
int    orc_huffman_lengths(const uint32_t freq[256], uint8_t lengths[256]);
void   orc_huffman_codes(const uint8_t lengths[256], uint32_t codes[256]);
int    orc_huffman_encode(const uint8_t* in, uint32_t n, orc_huffman_meta_t* meta, uint8_t** payload);
int    orc_huffman_decode(const orc_huffman_meta_t* meta, const uint8_t* data, uint8_t* out);
int    orc_encode_block(const uint8_t* in, uint32_t n, uint32_t* primary_index, orc_huffman_meta_t* meta, uint8_t** payload,
                        uint8_t* bwt_out, uint8_t* mtf_out, uint8_t** rle_out, size_t* rle_size);
uint32_t orc_crc32c(const void* data, uint64_t length, uint32_t previous_crc);
uint32_t orc_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint32_t len_b);
uint32_t orc_chunks_crc32c(const uint8_t* headers, const uint8_t* data, uint64_t total, uint32_t chunk_size, uint32_t crc);
uint32_t orc_entry_crc32c(uint32_t me_crc, int64_t tmpfile_size, uint32_t chunks_crc, uint64_t data_size);
size_t   orc_frame_record(const uint8_t header268[268], const uint8_t* payload, uint32_t encoded_size, uint8_t* out);
void   orc_free(void* p);

#ifdef __cplusplus
}
#endif
