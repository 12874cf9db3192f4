// Device check of bra::xlane<LM> (lane-exchange helpers) -- run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -I br-archive_amd/csrc scripts/xlane_check.hip -o /tmp/xl && /tmp/xl
#include "bra_hip_common.h"
#include <cstdio>

__global__ void k(uint32_t* out)
{
    const uint32_t l = threadIdx.x;
    out[0 * 64 + l]  = bra::xlane<1>(l * 3 + 1);
    out[1 * 64 + l]  = bra::xlane<2>(l * 3 + 1);
    out[2 * 64 + l]  = bra::xlane<4>(l * 3 + 1);
    out[3 * 64 + l]  = bra::xlane<8>(l * 3 + 1);
    out[4 * 64 + l]  = bra::xlane<16>(l * 3 + 1);
    out[5 * 64 + l]  = bra::xlane<32>(l * 3 + 1);
}

int main()
{
    uint32_t* d;
    uint32_t  h[6 * 64];
    (void) hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    (void) hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int m = 0; m < 6; ++m)
        for (uint32_t l = 0; l < 64; ++l)
            if (h[m * 64 + l] != ((l ^ (1u << m)) * 3 + 1))
            {
                if (bad++ < 10)
                    printf("LM %d lane %u got %u want %u\n", 1 << m, l, h[m * 64 + l], (l ^ (1u << m)) * 3 + 1);
            }
    printf(bad ? "xlane FAIL (%d)\n" : "xlane OK\n", bad);
    return bad != 0;
}
