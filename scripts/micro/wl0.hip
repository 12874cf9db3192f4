// Wide level-0 scatter micro-benchmark (measurement only, not product code).
// Question: what does placing every rotation of a block directly at its 16-bit-prefix sub-bucket
// cost, when a workgroup owns a part of the block's 65536 prefix bins and hands out slots from LDS
// running counters (unstaged 8-byte payload stores + the next digit byte)?  Compare with the
// current 8-bit level 0 + level-1 scatter (0.90 + 0.88 ms per 256 MiB of text, round 4).
//   parts P: the workgroups of one block each own 65536 / P bins (d0 ranges), all on one XCD.
#include <hip/hip_runtime.h>
#include <cstdint>

extern "C" __global__ void __launch_bounds__(1024) k_wl0(const uint8_t* __restrict__ in, const uint8_t* __restrict__ rank, uint32_t n,
                                                         uint32_t nblocks, const uint32_t* __restrict__ starts, uint64_t* __restrict__ opay,
                                                         uint8_t* __restrict__ odig, uint32_t P)
{
    extern __shared__ uint32_t run[];
    __shared__ uint8_t rk[256];
    const uint32_t w = blockIdx.x, x = w & 7, g = w >> 3;
    const uint32_t t = (g / P) * 8 + x, p = g % P;  // tile t on XCD t % 8, part p
    if (t >= nblocks)
        return;
    const uint32_t nb = 65536 / P, lo = p * nb;
    if (threadIdx.x < 256)
        rk[threadIdx.x] = rank[threadIdx.x];
    for (uint32_t i = threadIdx.x; i < nb; i += 1024)
        run[i] = starts[(size_t) t * 65536 + lo + i];
    __syncthreads();
    const uint8_t* b = in + (size_t) t * n;
    for (uint32_t e0 = threadIdx.x * 4; e0 < n; e0 += 4096)
    {
        const uint32_t q = *reinterpret_cast<const uint32_t*>(b + e0);
        const uint32_t q2 = *reinterpret_cast<const uint32_t*>(b + ((e0 + 4) % n));
        uint32_t c[8];
#pragma unroll
        for (int k = 0; k < 4; ++k)
        {
            c[k]     = rk[(q >> (8 * k)) & 0xFF];
            c[k + 4] = rk[(q2 >> (8 * k)) & 0xFF];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
        {
            const uint32_t d16 = (c[k] << 11) | (c[k + 1] << 6) | (c[k + 2] << 1) | (c[k + 3] >> 4);
            if (d16 - lo < nb)
            {
                const uint32_t slot = atomicAdd(&run[d16 - lo], 1u);
                opay[slot]          = ((uint64_t) d16 << 40) | ((uint64_t) c[k + 4] << 32) | (e0 + k);
                odig[slot]          = (uint8_t) ((c[k + 3] << 4) | (c[k + 4] >> 1));
            }
        }
    }
}

extern "C" int wl0_launch(const void* in, const void* rank, uint32_t n, uint32_t nblocks, const void* starts, void* opay, void* odig, uint32_t P,
                          void* stream)
{
    const uint32_t groups = (nblocks + 7) / 8;
    hipLaunchKernelGGL(k_wl0, dim3(groups * 8 * P), dim3(1024), (65536 / P) * 4, (hipStream_t) stream, (const uint8_t*) in, (const uint8_t*) rank,
                       n, nblocks, (const uint32_t*) starts, (uint64_t*) opay, (uint8_t*) odig, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int wl0_set_attr()
{
    return hipFuncSetAttribute((const void*) k_wl0, hipFuncAttributeMaxDynamicSharedMemorySize, 131072) == hipSuccess ? 0 : -1;
}
