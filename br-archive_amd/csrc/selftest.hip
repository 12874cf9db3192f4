// selftest.hip -- device self-test of the wave / workgroup scan primitives (bra_hip_common.h).
//
// Diagnostics only (not on the codec path): every primitive is run on several deterministic input
// patterns and compared with a serial restatement computed by one thread from LDS.  An error in a
// lane-exchange primitive can stay invisible in the codec's outputs (a wrong group boundary in the
// job kernels only costs an extra refinement round), so it is tested directly.
#include "bra_hip_common.h"
#include "../../include/bra_hip.h"

namespace bra {

namespace {

__device__ __forceinline__ uint32_t st_hash(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// One workgroup of 256 threads per pattern.  err[0] accumulates mismatches.
__global__ void __launch_bounds__(256) k_selftest(uint32_t* __restrict__ err)
{
    __shared__ uint32_t in[1024], out[1024];
    __shared__ uint32_t tmp[8];
    const uint32_t pat = blockIdx.x, t = threadIdx.x, lane = (uint32_t) lane_id(), w = t >> 6;
    // pattern: small values (sums stay in 32 bits), sparse values (max / min scans with ties)
    auto val = [&](uint32_t i) -> uint32_t {
        const uint32_t h = st_hash(i * 2654435761u + pat * 97u + 1u);
        return (pat & 1) ? ((h & 7u) == 0 ? (h >> 8) & 0xFFFFu : 0u) : (h & 0xFFu);
    };
    uint32_t bad = 0;
    // ---- wave_scan<FWD / reverse> on one value per lane, three operators ----
    const uint32_t x = val(t);
    const uint32_t sa = wave_scan<true>(x, 0u, OpAdd()), sm = wave_scan<true>(x, 0u, OpMax()), sn = wave_scan<true>(x, ~0u, OpMin());
    const uint32_t ra = wave_scan<false>(x, 0u, OpAdd()), rm = wave_scan<false>(x, 0u, OpMax()), rn = wave_scan<false>(x, ~0u, OpMin());
    {
        uint32_t ea = 0, em = 0, en = ~0u, fa = 0, fm = 0, fn = ~0u;
        for (uint32_t l = 0; l <= lane; ++l)
        {
            const uint32_t v = val(w * 64 + l);
            ea += v, em = max(em, v), en = min(en, v);
        }
        for (uint32_t l = lane; l < 64; ++l)
        {
            const uint32_t v = val(w * 64 + l);
            fa += v, fm = max(fm, v), fn = min(fn, v);
        }
        bad += (sa != ea) + (sm != em) + (sn != en) + (ra != fa) + (rm != fm) + (rn != fn);
    }
    // ---- 4-per-lane wave scans (element e = lane * 4 + r of this wave) ----
    uint32_t v4[4], e4[4], tot = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        v4[r] = val(1000 + w * 256 + lane * 4 + r);
    {
        uint32_t a[4] = {v4[0], v4[1], v4[2], v4[3]};
        wave_max_scan4(a);
        uint32_t b[4] = {v4[0], v4[1], v4[2], v4[3]};
        wave_min_rscan4(b);
        uint32_t c[4], d[4];
        wave_excl_sum4(v4, c, &tot);
        wave_excl_max4(v4, d);
        uint32_t run_max = 0, run_sum = 0, all = 0;
        for (uint32_t e = 0; e < 256; ++e)
            all += val(1000 + w * 256 + e);
        for (uint32_t e = 0; e < lane * 4; ++e)
        {
            const uint32_t v = val(1000 + w * 256 + e);
            run_max = max(run_max, v), run_sum += v;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
            const uint32_t e = lane * 4 + r;
            uint32_t       suf = ~0u;
            for (uint32_t q = e; q < 256; ++q)
                suf = min(suf, val(1000 + w * 256 + q));
            bad += (c[r] != run_sum) + (d[r] != run_max);
            run_max = max(run_max, v4[r]);
            run_sum += v4[r];
            bad += (a[r] != run_max) + (b[r] != suf);
        }
        bad += (tot != all);
    }
    // ---- block256_exclusive_sum ----
    in[t] = x;
    __syncthreads();
    uint32_t btot;
    const uint32_t bex = block256_exclusive_sum(x, tmp, &btot);
    out[t]             = bex;
    __syncthreads();
    if (t == 0)
    {
        uint32_t run = 0;
        for (uint32_t i = 0; i < 256; ++i)
        {
            bad += (out[i] != run);
            run += in[i];
        }
        bad += (btot != run);
    }
    if (bad)
        atomicAdd(err, bad);
}

}  // namespace

}  // namespace bra

extern "C" int bra_gpu_selftest(void)
{
    uint32_t* d = nullptr;
    uint32_t  h = 0;
    if (hipMalloc(&d, 4) != hipSuccess)
        return -1;
    int rc = -1;
    if (hipMemset(d, 0, 4) == hipSuccess)
    {
        hipLaunchKernelGGL(bra::k_selftest, dim3(8), dim3(256), 0, 0, d);
        if (hipGetLastError() == hipSuccess && hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost) == hipSuccess)
            rc = (int) std::min<uint32_t>(h, 0x7FFFFFFF);
    }
    (void) hipFree(d);
    return rc;
}
