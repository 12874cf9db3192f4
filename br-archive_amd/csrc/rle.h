// rle.h -- PackBits RLE stage (device pointers).
#pragma once

#include "mtf.h"  // Tiling, Piece

namespace bra {

constexpr uint32_t RLE_TILE = 4096;

// Worst-case RLE output of an n-byte block (all literals): n + ceil(n/128).
__host__ __device__ inline uint64_t rle_capacity(uint32_t n) { return (uint64_t) n + (n + 127) / 128 + 16; }

struct RleWorkspace
{
    Tiling   tiling;
    void*    runs = nullptr;
    void*    link = nullptr;
    void*    gaps = nullptr;
    void*    offs = nullptr;
    uint32_t cap  = 0;
    void*    dmap = nullptr;  // decode: segment entry maps and segment states
    uint64_t dmap_cap = 0;
    bool     reserve(uint32_t ntiles);
    bool     reserve_decode(uint64_t bytes);
    void     release();
};

// Encode every block of d_in (geometry h_blocks) into d_out at d_rle_base[b]; per-block output
// sizes to d_rle_size, byte histograms of the output to d_hist[b * 256 + c].
bool rle_encode_device(RleWorkspace& w, const uint8_t* d_in, const BlockDesc* h_blocks, uint32_t nblocks, const uint64_t* d_rle_base,
                       uint8_t* d_out, uint32_t* d_rle_size, uint32_t* d_hist, hipStream_t s);

// Decode: block b's stream is at d_in + d_in_base[b] (d_in_size[b] bytes; h_in_size: the same
// sizes on the host, used to split long streams into segments decoded in parallel); output goes to
// d_out + d_out_base[b] (capacity d_out_cap[b]; writes past it are dropped).  d_out_size[b] =
// decoded size, 0 on a malformed stream (bra_rle_decode_compute_size semantics).
bool rle_decode_device(RleWorkspace& w, const uint32_t* h_in_size, const uint8_t* d_in, const uint64_t* d_in_base, const uint32_t* d_in_size, uint32_t nblocks, uint8_t* d_out,
                       const uint64_t* d_out_base, const uint64_t* d_out_cap, uint32_t* d_out_size, hipStream_t s);

}  // namespace bra
