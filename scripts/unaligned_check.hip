// Checks that a global_load_dwordx4 from a byte address that is not 16-byte aligned returns the 16
// bytes at that address (hardware unaligned-access mode), and times aligned-pair vs single loads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

__global__ void k_unaligned(const uint8_t* __restrict__ in, const uint32_t* __restrict__ pos, uint32_t n, uint4* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
    {
        const uint8_t* p = in + pos[i];
        uint4 q;
        asm volatile("global_load_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(q) : "v"(p) : "memory");
        out[i] = q;
    }
}

int main()
{
    const uint32_t N = 1 << 20, M = 1 << 16;
    std::vector<uint8_t> h(N + 64);
    for (auto& c : h) c = (uint8_t) rand();
    std::vector<uint32_t> pos(M);
    for (auto& p : pos) p = (uint32_t) rand() % N;
    uint8_t* d_in; uint32_t* d_pos; uint4* d_out;
    hipMalloc(&d_in, N + 64); hipMalloc(&d_pos, M * 4); hipMalloc(&d_out, M * 16);
    hipMemcpy(d_in, h.data(), N + 64, hipMemcpyHostToDevice);
    hipMemcpy(d_pos, pos.data(), M * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_unaligned, dim3(M / 256), dim3(256), 0, 0, d_in, d_pos, M, d_out);
    hipError_t e = hipDeviceSynchronize();
    std::vector<uint8_t> o(M * 16);
    hipMemcpy(o.data(), d_out, M * 16, hipMemcpyDeviceToHost);
    int bad = 0;
    for (uint32_t i = 0; i < M; ++i)
        for (int b = 0; b < 16; ++b)
            if (o[i * 16 + b] != h[pos[i] + b]) { if (bad < 5) printf("mismatch i=%u pos=%u b=%d got %02x want %02x\n", i, pos[i], b, o[i*16+b], h[pos[i]+b]); ++bad; }
    printf("sync=%s unaligned dwordx4: %d bad of %u\n", hipGetErrorString(e), bad, M);
    return bad != 0;
}
