// bwt_large.hip -- BWT of one block of 2^24 bytes or more (the single-block C-ABI bra_bwt_encode2,
// /root/reference/src/encoders/bra_bwt.c:73-108, takes any u32 length; the batched MSD/job path
// packs 24-bit rotation indices into its payloads and stops at 2^24).
//
// Prefix doubling over cyclic rotations: after the pass with offset h every rotation carries the
// rank of its first 2h bytes (the number of rotations whose first 2h bytes are smaller).  A pass
// builds key(i) = rank(i) << B | rank((i + h) mod n), B = ceil(log2 n) bits, for i in index order,
// radix-sorts (key, i) pairs with rocPRIM (stable: tied rotations stay in index order, the glibc
// qsort_r merge-sort tie rule of the reference), and assigns each rotation the start of its key's
// run (head flags + max-scan).  It stops once every key is distinct or 2h >= n (identical rotations
// of a periodic block).  L[j] = in[(sa[j] + n - 1) mod n], pi = the slot holding rotation 0.
// HBM traffic per pass ~ (8 + 4) B written / read per element by the sort's ceil(2B / 8) digit
// passes plus 32 B for the key build, the head scan and the rank scatter; text blocks of 16-64 MiB
// finish in 6-10 passes.  This path is for correctness at large sizes, not the benchmark shape.
#include "bwt.h"

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

namespace bra {
namespace {

// pass 0: key(i) = in[i] << B | in[(i + 1) mod n] (the first two bytes of rotation i)
__global__ void k_lg_keys0(const uint8_t* __restrict__ in, uint32_t n, uint32_t B, uint64_t* __restrict__ key, uint32_t* __restrict__ idx)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    {
        const uint32_t j = i + 1 == n ? 0u : i + 1;
        key[i]           = ((uint64_t) in[i] << B) | in[j];
        idx[i]           = i;
    }
}

// pass h: key(i) = rank[i] << B | rank[(i + h) mod n]
__global__ void k_lg_keys(const uint32_t* __restrict__ rank, uint32_t n, uint32_t h, uint32_t B, uint64_t* __restrict__ key,
                          uint32_t* __restrict__ idx)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    {
        const uint64_t j = (uint64_t) i + h;
        key[i]           = ((uint64_t) rank[i] << B) | rank[j >= n ? j - n : j];
        idx[i]           = i;
    }
}

// head[j] = j at the start of a run of equal keys, else 0; *tied = 1 if any run has length > 1
__global__ void k_lg_heads(const uint64_t* __restrict__ key, uint32_t n, uint32_t* __restrict__ head, uint32_t* __restrict__ tied)
{
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    {
        const bool h = j == 0 || key[j] != key[j - 1];
        head[j]      = h ? j : 0u;
        if (!h)
            *tied = 1u;  // plain vector store; every writer stores the same value
    }
}

__global__ void k_lg_rank(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ grp, uint32_t n, uint32_t* __restrict__ rank)
{
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
        rank[sa[j]] = grp[j];
}

__global__ void k_lg_emit(const uint8_t* __restrict__ in, const uint32_t* __restrict__ sa, uint32_t n, uint8_t* __restrict__ L,
                          uint32_t* __restrict__ pi)
{
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    {
        const uint32_t r = sa[j];
        L[j]             = in[r == 0 ? n - 1 : r - 1];
        if (r == 0)
            *pi = j;
    }
}

template <typename T>
struct DevBuf
{
    T* p = nullptr;
    ~DevBuf() { (void) hipFree(p); }
    bool alloc(size_t n) { return hipMalloc((void**) &p, n * sizeof(T) + 16) == hipSuccess; }
};

}  // namespace

bool bwt_encode_large(const uint8_t* d_in, uint32_t n, uint8_t* d_L, uint32_t* d_pi, hipStream_t s)
{
    if (n < 2)
    {
        if (n == 0)
            return false;
        return hipMemcpyAsync(d_L, d_in, 1, hipMemcpyDeviceToDevice, s) == hipSuccess && hipMemsetAsync(d_pi, 0, 4, s) == hipSuccess &&
               hipStreamSynchronize(s) == hipSuccess;
    }
    uint32_t B = 8;
    while (B < 32 && (1ull << B) < n)
        ++B;
    DevBuf<uint64_t> k0, k1;
    DevBuf<uint32_t> i0, sa, rank, grp, flag;
    if (!k0.alloc(n) || !k1.alloc(n) || !i0.alloc(n) || !sa.alloc(n) || !rank.alloc(n) || !grp.alloc(n) || !flag.alloc(1))
    {
        bra_hip_report("bwt: large block of %u bytes: device allocation failed", n);
        return false;
    }
    size_t sort_bytes = 0, scan_bytes = 0;
    if (rocprim::radix_sort_pairs(nullptr, sort_bytes, k0.p, k1.p, i0.p, sa.p, (size_t) n, 0u, 2 * B, s) != hipSuccess ||
        rocprim::inclusive_scan(nullptr, scan_bytes, grp.p, grp.p, (size_t) n, rocprim::maximum<uint32_t>(), s) != hipSuccess)
        return false;
    DevBuf<uint8_t> tmp;
    if (!tmp.alloc(std::max(sort_bytes, scan_bytes)))
    {
        bra_hip_report("bwt: large block of %u bytes: device allocation failed", n);
        return false;
    }
    const dim3 grid(std::min<uint32_t>(div_up(n, 256), 65536u)), tpb(256);
    for (uint64_t h = 0;; h = h ? 2 * h : 2)
    {
        // h = 0: the first two bytes; afterwards ranks cover h bytes and the key covers 2h
        if (h == 0)
            hipLaunchKernelGGL(k_lg_keys0, grid, tpb, 0, s, d_in, n, B, k0.p, i0.p);
        else
            hipLaunchKernelGGL(k_lg_keys, grid, tpb, 0, s, rank.p, n, (uint32_t) h, B, k0.p, i0.p);
        size_t sb = sort_bytes, cb = scan_bytes;
        if (rocprim::radix_sort_pairs(tmp.p, sb, k0.p, k1.p, i0.p, sa.p, (size_t) n, 0u, 2 * B, s) != hipSuccess)
            return false;
        const uint64_t covered = h ? 2 * h : 2;  // bytes of each rotation the sorted keys compare
        if (covered >= n)
            break;  // whole rotations compared: remaining ties are identical rotations (index order)
        if (hipMemsetAsync(flag.p, 0, 4, s) != hipSuccess)
            return false;
        hipLaunchKernelGGL(k_lg_heads, grid, tpb, 0, s, k1.p, n, grp.p, flag.p);
        if (rocprim::inclusive_scan(tmp.p, cb, grp.p, grp.p, (size_t) n, rocprim::maximum<uint32_t>(), s) != hipSuccess)
            return false;
        hipLaunchKernelGGL(k_lg_rank, grid, tpb, 0, s, sa.p, grp.p, n, rank.p);
        uint32_t tied = 0;
        if (hipMemcpyAsync(&tied, flag.p, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return false;
        if (!tied)
            break;  // every rotation's rank is final
    }
    hipLaunchKernelGGL(k_lg_emit, grid, tpb, 0, s, d_in, sa.p, n, d_L, d_pi);
    return hipStreamSynchronize(s) == hipSuccess && hipGetLastError() == hipSuccess;
}

}  // namespace bra
