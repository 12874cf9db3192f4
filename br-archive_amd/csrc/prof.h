// prof.h -- optional per-kernel timing with HIP events (bench.py reads it through the C-ABI).
// Off unless a context enables it; when on, an event pair is recorded around every launch of the
// enabled slots on the launch's own stream.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace bra {

enum ProfSlot : int
{
    P_STAGE_BWT, P_STAGE_MTF, P_STAGE_RLE, P_STAGE_HUF,
    P_BWT_L0HIST, P_BWT_L0SCATTER, P_BWT_PACK, P_BWT_HIST, P_BWT_SCAN, P_BWT_SCATTER, P_BWT_JOBS, P_BWT_MJOBS, P_BWT_FALLBACK,
    P_MTF_LASTOCC, P_MTF_SCAN, P_MTF_ENCODE,
    P_RLE_RUNS, P_RLE_LINK, P_RLE_SIZES, P_RLE_OFFSETS, P_RLE_WRITE,
    P_HUF_BUILD, P_HUF_OFFSETS, P_HUF_TILEBITS, P_HUF_TILESCAN, P_HUF_ZERO, P_HUF_PACK,
    P_FRAME, P_CRC,
    P_DEC_HUF, P_DEC_RLE, P_DEC_MTF, P_DEC_IBWT,       // decode stages
    P_DEC_HD_TRANS, P_DEC_RLED, P_DEC_MTF_LOCAL, P_DEC_IB_WALK,  // their largest kernels
    P_DEC_IB_PAIR,
    P_NSLOT
};

const char* prof_name(int slot);

struct Prof
{
    uint64_t                                            mask = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>>      pending[P_NSLOT];
    std::vector<hipEvent_t>                             pool;
    double                                              ms[P_NSLOT] = {};
    uint32_t                                            launches[P_NSLOT] = {};
    double                                              bytes[P_NSLOT] = {};  // algorithmic bytes of the timed launches
    hipEvent_t                                          get();
    void                                                collect();  // waits for the recorded events
    void                                                reset();
    ~Prof();
};

// Set by the C-ABI for the duration of a call, per calling thread: contexts used from several
// threads (or on several devices) each time only their own launches.
extern thread_local Prof* g_prof;

// Attribute algorithmic bytes ("algorithmic bytes") to a slot's timed launches.
inline void prof_bytes(int slot, double b)
{
    if (g_prof && (g_prof->mask >> slot & 1))
        g_prof->bytes[slot] += b;
}

struct ProfScope
{
    int         slot;
    hipStream_t s;
    hipEvent_t  e0 = nullptr;
    ProfScope(int slot_, hipStream_t s_) : slot(slot_), s(s_)
    {
        if (g_prof && (g_prof->mask >> slot & 1))
        {
            e0 = g_prof->get();
            (void) hipEventRecord(e0, s);
        }
    }
    ~ProfScope()
    {
        if (e0)
        {
            hipEvent_t e1 = g_prof->get();
            (void) hipEventRecord(e1, s);
            g_prof->pending[slot].push_back({e0, e1});
        }
    }
};

}  // namespace bra

#define BRA_PROF(slot, stream) ::bra::ProfScope _bra_prof_##slot(::bra::slot, stream)
