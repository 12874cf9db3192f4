// ibwt.h -- inverse BWT stage (device pointers).
#pragma once

#include "mtf.h"  // Tiling

namespace bra {

struct IbwtWorkspace
{
    Tiling    tiling;
    uint32_t* T        = nullptr;  // transform, block-local indices
    uint64_t* T2       = nullptr;  // main path: two transform steps per entry (k_ib_pair)
    uint64_t  cap_n2   = 0;
    uint32_t* th       = nullptr;
    uint32_t* hop_next = nullptr;
    uint32_t* hop_len  = nullptr;
    uint32_t* start    = nullptr;
    uint32_t* cyc      = nullptr;
    uint32_t* nopair   = nullptr;  // blocks unsuited to the two-step walk (k_ib_scan)
    uint64_t  cap_n    = 0;
    uint32_t  cap_t = 0, cap_b = 0;
    // main path (ibwt.hip): block records, splitter prefix, control words, hops, staging
    uint64_t*              blk = nullptr;
    uint32_t*              cum = nullptr;
    uint32_t*              ctl = nullptr;
    uint32_t *             m_next = nullptr, *m_len = nullptr, *m_ovf = nullptr, *m_start = nullptr, *ovl_next = nullptr;
    uint32_t *             m_order = nullptr, *m_cnt = nullptr;  // hops in output order, chain hops per block
    uint8_t *              slot = nullptr, *pool = nullptr;
    uint32_t               cap_mb = 0, cap_ms = 0, pool_cap = 0, G = 0, walk_wg = 384;
    bool                   pair = false;  // two-step walk (k_ib_pair)
    uint64_t               cap_slot = 0;
    std::vector<uint64_t>  h_blk;
    std::vector<uint32_t>  h_ctl;
    std::vector<BlockDesc> h_key;
    bool                   reserve(uint64_t n, uint32_t nblocks, uint32_t ntiles);
    bool                   reserve_main(uint32_t nblocks, uint32_t nsplit, uint64_t slot_bytes);
    void                   release();
};

// keep_transform: leave the reference's transform (block-local u32 indices) in w.T.
bool ibwt_device(IbwtWorkspace& w, const uint8_t* d_L, const uint32_t* d_pi, const BlockDesc* d_blocks, const BlockDesc* h_blocks,
                 uint32_t nblocks, uint8_t* d_out, hipStream_t s, bool keep_transform = false);

}  // namespace bra
