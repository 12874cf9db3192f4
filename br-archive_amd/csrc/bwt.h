// bwt.h -- device-side stage entry points of the block codec (host-callable, device pointers).
#pragma once

#include "bra_hip_common.h"

namespace bra {

struct BwtWorkspace;
BwtWorkspace* bwt_workspace_create();
void          bwt_workspace_destroy(BwtWorkspace* w);

// Per block (after bwt_encode_device): 256-bit presence mask of its byte values, 8 dwords each (the
// BWT output has the same bytes, so the MTF stage takes its alphabets from here).
const uint32_t* bwt_alpha_masks(const BwtWorkspace* w);
// The suffix-array slots of the last encode (u32 per element at the block offsets; diagnostics).
const uint32_t* bwt_sa(const BwtWorkspace* w);
// Diagnostics: re-run the last STRING encode's job phase `reps` times (inputs reordered when
// shuffle_seed != 0) and audit every run; returns the failing jobs summed over the runs (-1: error).
// Valid only right after an encode whose input the caller still holds; -1 otherwise.
int  bwt_debug_rerun_jobs(BwtWorkspace* w, int reps, hipStream_t s, uint32_t shuffle_seed);
void bwt_forget_jobs(BwtWorkspace* w);  // any other call on the context invalidates the re-run state

// BWT of every block: d_L[off..off+len) = last column, d_pi[b] = primary index (block-local).
bool bwt_encode_device(BwtWorkspace* w, const uint8_t* d_in, const BlockDesc* d_blocks, const BlockDesc* h_blocks, uint32_t nblocks,
                       uint8_t* d_L, uint32_t* d_pi, hipStream_t s);
// The same in two halves: _enqueue queues everything up to the jobs without waiting for them;
// _finish waits for the jobs' mailbox and, when groups are still tied (periodic or highly repetitive
// blocks), runs the prefix-doubling fallback, which rewrites those blocks' L and pi on the stream
// (*fallback_ran tells the caller that work it queued in between read the earlier L).
bool bwt_encode_enqueue(BwtWorkspace* w, const uint8_t* d_in, const BlockDesc* d_blocks, const BlockDesc* h_blocks, uint32_t nblocks,
                        uint8_t* d_L, uint32_t* d_pi, hipStream_t s);
bool bwt_encode_finish(BwtWorkspace* w, const uint8_t* d_in, const BlockDesc* d_blocks, const BlockDesc* h_blocks, uint32_t nblocks,
                       uint8_t* d_L, uint32_t* d_pi, hipStream_t s, bool* fallback_ran);

// BWT of one block of any length >= 1 (bwt_large.hip: prefix doubling over cyclic rotations, the
// (key, index) pairs sorted by a hand-written stable LSD radix sort), used by the single-block C-ABI
// for blocks of 2^24 bytes or more; synchronises the stream.
bool bwt_encode_large(const uint8_t* d_in, uint32_t n, uint8_t* d_L, uint32_t* d_pi, hipStream_t s);

}  // namespace bra
