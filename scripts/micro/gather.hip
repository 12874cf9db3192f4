// Micro-benchmark (measurement only, not product): cost of one random 16-byte gather per lane from a
// 224 MiB byte string, by address alignment and load form -- the shape of the job kernels' round-1
// gather (pk_load128) and the MSD scatters' 8-byte digit loads (pk_load64).
//   mode 0: uint4 at a byte address (unaligned, as pk_load128)
//   mode 1: uint4 at the address rounded down to 4 bytes
//   mode 2: uint4 at the address rounded down to 16 bytes
//   mode 3: two uint2 at the address rounded down to 8 bytes (+0, +8)
//   mode 4: uint2 at a byte address (unaligned, as pk_load64)
//   mode 5: uint2 at the address rounded down to 8 bytes
//   mode 6: three uint2 at the address rounded down to 8 bytes (covers 16 bytes from any byte)
// Each lane handles 4 gathers (like a job lane's 4 slots), indices read coalesced.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint4 __attribute__((aligned(1))) uint4_u;
typedef uint2 __attribute__((aligned(1))) uint2_u;

__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ s, const uint32_t* __restrict__ idx, uint64_t n,
                                                int mode, uint32_t* __restrict__ out)
{
    const uint64_t base = ((uint64_t) blockIdx.x * 256 + threadIdx.x) * 4;
    if (base >= n)
        return;
    uint32_t acc = 0;
    uint32_t p[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
        p[r] = idx[base + r];
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
        const uint32_t a = p[r];
        switch (mode)
        {
        case 0: { const uint4 q = *reinterpret_cast<const uint4_u*>(s + a); acc += q.x ^ q.y ^ q.z ^ q.w; break; }
        case 1: { const uint4 q = *reinterpret_cast<const uint4*>(s + (a & ~3u)); acc += q.x ^ q.y ^ q.z ^ q.w; break; }
        case 2: { const uint4 q = *reinterpret_cast<const uint4*>(s + (a & ~15u)); acc += q.x ^ q.y ^ q.z ^ q.w; break; }
        case 3:
        {
            const uint2 q0 = *reinterpret_cast<const uint2*>(s + (a & ~7u));
            const uint2 q1 = *reinterpret_cast<const uint2*>(s + (a & ~7u) + 8);
            acc += q0.x ^ q0.y ^ q1.x ^ q1.y;
            break;
        }
        case 4: { const uint2 q = *reinterpret_cast<const uint2_u*>(s + a); acc += q.x ^ q.y; break; }
        case 5: { const uint2 q = *reinterpret_cast<const uint2*>(s + (a & ~7u)); acc += q.x ^ q.y; break; }
        default:
        {
            const uint2 q0 = *reinterpret_cast<const uint2*>(s + (a & ~7u));
            const uint2 q1 = *reinterpret_cast<const uint2*>(s + (a & ~7u) + 8);
            const uint2 q2 = *reinterpret_cast<const uint2*>(s + (a & ~7u) + 16);
            acc += q0.x ^ q0.y ^ q1.x ^ q1.y ^ q2.x ^ q2.y;
            break;
        }
        }
    }
    out[base / 4] = acc;
}

extern "C" int gather_run(const uint8_t* s, const uint32_t* idx, uint64_t n, int mode, uint32_t* out, int reps, float* ms)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const unsigned grid = (unsigned) ((n / 4 + 255) / 256);
    hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, 0, s, idx, n, mode, out);
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, 0, s, idx, n, mode, out);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(ms, e0, e1);
    *ms /= reps;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return (int) hipGetLastError();
}
