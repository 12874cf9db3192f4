// huffman.h -- canonical Huffman stage (device pointers).
#pragma once

#include "rle.h"

namespace bra {

// Same layout as the reference's packed bra_huffman_t (src/lib_bra_types.h:51-56).
#pragma pack(push, 1)
struct HuffMetaRec
{
    uint8_t  lengths[256];
    uint32_t orig_size;
    uint32_t encoded_size;
};
#pragma pack(pop)
static_assert(sizeof(HuffMetaRec) == 264, "bra_huffman_t layout");

struct HuffWorkspace
{
    Tiling    tiling;
    uint32_t* codes      = nullptr;
    uint32_t* tbits      = nullptr;
    uint64_t* tbit0      = nullptr;
    int32_t*  tree_child = nullptr;
    uint8_t*  tree_sym   = nullptr;
    uint32_t* table      = nullptr;
    uint32_t* status     = nullptr;
    void*     seg        = nullptr;  // segment-parallel decode: 3 x cap_seg segment records
    uint32_t* seg_off    = nullptr;
    uint32_t* seg_base   = nullptr;
    uint64_t* end_pos    = nullptr;
    uint32_t* flag       = nullptr;
    uint32_t* h_flag     = nullptr;  // pinned: flag, then the segment bases
    uint32_t  cap_b = 0, cap_t = 0, cap_tree = 0, cap_seg = 0, cap_segb = 0;
    // canonical fast path: per-block tables, per-segment transfer words, WG tasks
    uint32_t*             tab   = nullptr;
    uint32_t*             trans = nullptr;
    uint32_t*             seg_info = nullptr;
    uint32_t*             bmbuf    = nullptr;  // per segment: the entry-0 path's boundary bitmap
    uint32_t*             tflag    = nullptr;  // per task: compute every entry; [ntasks]: the chain's redo flag
    void*                 tasks = nullptr;
    uint32_t              cap_fb = 0, cap_fs = 0, cap_ft = 0;
    std::vector<uint32_t> h_segb;
    bool      reserve(uint32_t nblocks, uint32_t ntiles);
    bool      reserve_fast(uint32_t nblocks, uint32_t nseg, uint32_t ntasks);
    bool      reserve_tree(uint32_t nblocks);
    bool      reserve_segs(uint32_t nseg, uint32_t nblocks);
    void      release();
};

// Encode block b's RLE output (at h_rle_cap_blocks[b].off, d_rle_size[b] bytes, byte histogram in
// d_hist) into d_payload at d_payload_off[b] (d_payload_off has nblocks+1 entries; the last one is
// the total, also returned in *h_total).  d_meta[b] receives the bra_huffman_t of the block.
bool huff_encode_device(HuffWorkspace& w, const uint8_t* d_rle, const BlockDesc* h_rle_cap_blocks, uint32_t nblocks, const uint32_t* d_hist,
                        const uint32_t* d_rle_size, HuffMetaRec* d_meta, uint64_t* d_payload_off, uint8_t* d_payload, uint64_t payload_cap,
                        uint64_t* h_total, hipStream_t s,
                        bool cap_sufficient = false);

// Decode every block: d_out + d_out_base[b] receives meta[b].orig_size bytes; d_status[b] != 0 on
// a stream the reference would reject.  h_encoded_size: host copy of meta[b].encoded_size.
bool huff_decode_device(HuffWorkspace& w, const HuffMetaRec* d_meta, const uint32_t* h_encoded_size, uint32_t nblocks, const uint8_t* d_payload,
                        const uint64_t* d_payload_off, uint8_t* d_out, const uint64_t* d_out_base, uint32_t* d_status, hipStream_t s);

// Byte histograms of blocks (d_hist[b * 256 + c]).
bool histogram_device(Tiling& tiling, const uint8_t* d_in, const BlockDesc* h_blocks, uint32_t nblocks, uint32_t* d_hist, hipStream_t s);

}  // namespace bra
