// valu_cal.hip -- calibration of the VALU issue counters (measurement only).
//
// Every wave runs ITERS iterations of 16 independent v_add_u32 (inline asm, so the instruction count
// is exact: 16 * ITERS per wave) at full occupancy (8 waves per SIMD, 256 threads per workgroup,
// 8 workgroups per CU).  The program prints the kernel time (HIP events) and the issue rate it
// implies: wave-instructions per SIMD per shader cycle at the clock the caller passes in (or at the
// clock derived from GRBM_GUI_ACTIVE in a --pmc pass of the same binary).  Run under
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
//   rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT
// to get the counters of a VALU-saturated kernel: bench.py scales the job kernels' counters by them.
//
//   hipcc --offload-arch=gfx950 -O3 valu_cal.hip -o valu_cal && ./valu_cal [iters] [wgs_per_cu]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(256) k_valu_cal(uint32_t iters, uint32_t* out)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t a8 = a0 + 8, a9 = a0 + 9, a10 = a0 + 10, a11 = a0 + 11, a12 = a0 + 12, a13 = a0 + 13, a14 = a0 + 14, a15 = a0 + 15;
    const uint32_t b = blockIdx.x | 1u;
    for (uint32_t i = 0; i < iters; ++i)
    {
        asm volatile(
            "v_add_u32 %0, %0, %16\n v_add_u32 %1, %1, %16\n v_add_u32 %2, %2, %16\n v_add_u32 %3, %3, %16\n"
            "v_add_u32 %4, %4, %16\n v_add_u32 %5, %5, %16\n v_add_u32 %6, %6, %16\n v_add_u32 %7, %7, %16\n"
            "v_add_u32 %8, %8, %16\n v_add_u32 %9, %9, %16\n v_add_u32 %10, %10, %16\n v_add_u32 %11, %11, %16\n"
            "v_add_u32 %12, %12, %16\n v_add_u32 %13, %13, %16\n v_add_u32 %14, %14, %16\n v_add_u32 %15, %15, %16\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+v"(a8), "+v"(a9), "+v"(a10), "+v"(a11),
              "+v"(a12), "+v"(a13), "+v"(a14), "+v"(a15)
            : "v"(b));
    }
    const uint32_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ a8 ^ a9 ^ a10 ^ a11 ^ a12 ^ a13 ^ a14 ^ a15;
    if (s == 0x12345678u)  // practically never: keeps the adds alive
        out[blockIdx.x] = s;
}

int main(int argc, char** argv)
{
    const uint32_t iters = argc > 1 ? (uint32_t) atoi(argv[1]) : 20000;
    const uint32_t wpc   = argc > 2 ? (uint32_t) atoi(argv[2]) : 8;
    int            dev = 0, cus = 0, clk_khz = 0;
    (void) hipGetDevice(&dev);
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void) hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
    const uint32_t grid = (uint32_t) cus * wpc;
    uint32_t*      out  = nullptr;
    if (hipMalloc(&out, grid * sizeof(uint32_t)) != hipSuccess)
        return 1;
    hipEvent_t e0, e1;
    (void) hipEventCreate(&e0);
    (void) hipEventCreate(&e1);
    k_valu_cal<<<grid, 256>>>(iters / 10, out);  // warm-up
    (void) hipEventRecord(e0);
    k_valu_cal<<<grid, 256>>>(iters, out);
    (void) hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess)
        return 1;
    float ms = 0;
    (void) hipEventElapsedTime(&ms, e0, e1);
    const double waves      = (double) grid * 4;
    const double wave_insts = waves * 16.0 * iters;
    const double simds      = (double) cus * 4;
    const double clk        = clk_khz * 1e3;
    printf("{\"kernel\": \"k_valu_cal\", \"cus\": %d, \"grid\": %u, \"waves_per_simd\": %.1f, \"iters\": %u, \"ms\": %.4f, "
           "\"valu_wave_insts\": %.6g, \"max_clock_hz\": %.6g, \"wave_insts_per_simd_per_cycle_at_max_clock\": %.4f}\n",
           cus, grid, waves / simds, iters, ms, wave_insts, clk, wave_insts / simds / (ms * 1e-3 * clk));
    (void) hipFree(out);
    return 0;
}
