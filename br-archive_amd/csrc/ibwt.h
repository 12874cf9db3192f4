// ibwt.h -- inverse BWT stage (device pointers).
#pragma once

#include "mtf.h"  // Tiling

namespace bra {

struct IbwtWorkspace
{
    Tiling    tiling;
    uint32_t* T        = nullptr;  // transform, block-local indices
    uint32_t* th       = nullptr;
    uint32_t* hop_next = nullptr;
    uint32_t* hop_len  = nullptr;
    uint32_t* start    = nullptr;
    uint32_t* cyc      = nullptr;
    uint64_t  cap_n    = 0;
    uint32_t  cap_t = 0, cap_b = 0;
    bool      reserve(uint64_t n, uint32_t nblocks, uint32_t ntiles);
    void      release();
};

bool ibwt_device(IbwtWorkspace& w, const uint8_t* d_L, const uint32_t* d_pi, const BlockDesc* d_blocks, const BlockDesc* h_blocks,
                 uint32_t nblocks, uint8_t* d_out, hipStream_t s);

}  // namespace bra
