// mtf.h -- move-to-front stage (device pointers) + the block tiling helper shared by the stages.
#pragma once

#include "bra_hip_common.h"

#include <algorithm>
#include <vector>

namespace bra {

// A fixed-size piece of one block (the last piece of a block may be short).
struct Piece
{
    uint64_t off;    // absolute offset of the piece in the batch buffer
    uint32_t start;  // offset inside its block
    uint32_t len;
    uint32_t block;
    uint32_t pad;
};

// Cut every block into pieces of `piece` bytes; device copies of the piece list and of the
// per-block (first piece, piece count).  Rebuilt only when the geometry changes.
struct Tiling
{
    uint32_t               n        = 0;
    Piece*                 d_pieces = nullptr;
    uint32_t*              d_first  = nullptr;
    uint32_t*              d_count  = nullptr;
    std::vector<Piece>     h_pieces;
    std::vector<uint32_t>  h_first, h_count;
    std::vector<BlockDesc> key;
    uint32_t               key_piece = 0;
    size_t                 cap_p = 0, cap_b = 0;

    bool build(const BlockDesc* blocks, uint32_t nblocks, uint32_t piece, hipStream_t s)
    {
        if (piece == key_piece && key.size() == nblocks &&
            std::equal(key.begin(), key.end(), blocks, [](const BlockDesc& a, const BlockDesc& b) { return a.off == b.off && a.len == b.len; }))
            return true;
        h_pieces.clear();
        h_first.assign(nblocks, 0);
        h_count.assign(nblocks, 0);
        for (uint32_t b = 0; b < nblocks; ++b)
        {
            h_first[b] = (uint32_t) h_pieces.size();
            for (uint32_t st = 0; st < blocks[b].len; st += piece)
                h_pieces.push_back(Piece{blocks[b].off + st, st, std::min(piece, blocks[b].len - st), b, 0});
            h_count[b] = (uint32_t) h_pieces.size() - h_first[b];
        }
        n = (uint32_t) h_pieces.size();
        key.clear();  // the cached geometry is valid only once the copies below have been issued
        if (n > cap_p)
        {
            cap_p          = 0;
            const size_t c = n + n / 4 + 16;
            if (!dev_alloc(d_pieces, c))
                return false;
            cap_p = c;
        }
        if (nblocks > cap_b)
        {
            cap_b          = 0;
            const size_t c = nblocks + 16;
            if (!dev_alloc(d_first, c) || !dev_alloc(d_count, c))
                return false;
            cap_b = c;
        }
        BRA_HIP_CHECK(hipMemcpyAsync(d_pieces, h_pieces.data(), n * sizeof(Piece), hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipMemcpyAsync(d_first, h_first.data(), nblocks * 4, hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipMemcpyAsync(d_count, h_count.data(), nblocks * 4, hipMemcpyHostToDevice, s));
        BRA_HIP_CHECK(hipStreamSynchronize(s));  // host vectors are the source of the async copies
        key.assign(blocks, blocks + nblocks);
        key_piece = piece;
        return true;
    }

    void release()
    {
        (void) hipFree(d_pieces);
        (void) hipFree(d_first);
        (void) hipFree(d_count);
        *this = Tiling{};
    }
};

constexpr uint32_t MTF_SEG     = 2048;  // symbols per thread-segment (decode)
constexpr uint32_t MTF_SEG_ENC = 1024;  // encode segments: twice the threads, for the register-table kernel
constexpr uint32_t MTF_REG     = 32;    // table entries the register kernel keeps (blocks of <= 32 distinct symbols)

struct MtfWorkspace
{
    Tiling    tiling;
    void*     state     = nullptr;
    size_t    cap_state = 0;
    uint32_t* nsym      = nullptr;  // distinct symbols per block (k_mtf_alpha)
    uint8_t*  amap      = nullptr;  // per block: alphabet index of every byte value (0xFF: absent)
    uint8_t*  ainv      = nullptr;  // per block: byte value of alphabet index a < 32 (position-table blocks)
    uint32_t* amode     = nullptr;  // per block: position-table dwords (4 / 8) of k_mtf_encode_pos, 0: other encoders
    uint32_t* amask     = nullptr;  // per block: presence mask (when the caller has none)
    uint32_t  cap_nsym  = 0;
    // chunks of half segments of the position-table passes (built with the tiling's geometry)
    uint32_t*             pt_chunk0 = nullptr;  // per block: first chunk
    uint32_t*             pt_chunk_blk = nullptr;  // per chunk: block
    int32_t*              pt_cmax = nullptr;   // per chunk: 32 maxima, then exclusive prefixes
    uint32_t              pt_nchunks = 0;
    size_t                pt_cap_c = 0, pt_cap_b = 0;
    std::vector<uint32_t> pt_key;              // per block segment counts the chunk arrays were built for

    bool reserve(size_t bytes)
    {
        if (bytes <= cap_state)
            return true;
        cap_state      = 0;
        const size_t c = bytes + bytes / 4 + 4096;
        if (!dev_alloc_bytes(state, c))
            return false;
        cap_state = c;
        return true;
    }
    bool reserve_blocks(uint32_t nblocks)
    {
        if (nblocks <= cap_nsym)
            return true;
        cap_nsym = 0;
        if (!dev_alloc(nsym, (uint64_t) nblocks + 64) || !dev_alloc(amap, 256ull * (nblocks + 64)) || !dev_alloc(amode, (uint64_t) nblocks + 64) ||
            !dev_alloc(ainv, 32ull * (nblocks + 64)) || !dev_alloc(amask, 8ull * (nblocks + 64)))
            return false;
        cap_nsym = nblocks + 64;
        return true;
    }
    void release()
    {
        tiling.release();
        (void) hipFree(state);
        (void) hipFree(nsym);
        (void) hipFree(amap);
        (void) hipFree(amode);
        (void) hipFree(ainv);
        (void) hipFree(amask);
        (void) hipFree(pt_chunk0);
        (void) hipFree(pt_chunk_blk);
        (void) hipFree(pt_cmax);
        pt_chunk0 = pt_chunk_blk = nullptr;
        pt_cmax                  = nullptr;
        pt_nchunks               = 0;
        pt_cap_c = pt_cap_b = 0;
        pt_key.clear();
        state     = nullptr;
        nsym      = nullptr;
        amap      = nullptr;
        amode     = nullptr;
        ainv      = nullptr;
        amask     = nullptr;
        cap_state = 0;
        cap_nsym  = 0;
    }
};

// d_amask: per block presence masks of d_in's blocks (8 dwords each, e.g. bwt_alpha_masks), or null.
bool mtf_encode_device(MtfWorkspace& w, const uint8_t* d_in, uint8_t* d_out, const BlockDesc* h_blocks, uint32_t nblocks, hipStream_t s,
                       const uint32_t* d_amask = nullptr);
// d_tmp: scratch of the batch size (labels)
bool mtf_decode_device(MtfWorkspace& w, const uint8_t* d_in, uint8_t* d_out, uint8_t* d_tmp, const BlockDesc* h_blocks, uint32_t nblocks,
                       hipStream_t s);

}  // namespace bra
