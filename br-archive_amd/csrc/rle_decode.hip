// rle_decode.hip -- PackBits decoding for a batch of independent blocks.
//
// Replaces bra_rle_decode / bra_rle_decode_compute_size (reference src/encoders/bra_rle.c:122-160,
// :162-224): control c >= 0 -> c+1 literal bytes follow; -127 <= c <= -1 -> the next byte repeated
// 1-c times; c == -128 -> no-op; a block truncated by the end of the stream makes the decoded size
// 0 (error).
//
// The position of each control byte depends on every earlier one, so one lane per block parses the
// control bytes out of an LDS window of the stream (the payload bytes are never touched) and
// records (stream offset, output offset) per control; all threads then expand the records.
#include "rle.h"

namespace bra {

namespace {

constexpr uint32_t WIN = 8192;

struct Rec
{
    uint32_t src, dst;
};

// one 64-thread workgroup per block
__global__ void __launch_bounds__(64) k_rled_parse(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_base,
                                                   const uint32_t* __restrict__ in_size, uint32_t nblocks, Rec* __restrict__ recs,
                                                   const uint64_t* __restrict__ rec_base, uint32_t* __restrict__ nrec,
                                                   uint32_t* __restrict__ out_size)
{
    __shared__ uint8_t  win[WIN];
    __shared__ uint32_t sh_i, sh_dst, sh_n, sh_err;
    for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    {
        const uint8_t* src  = in + in_base[b];
        const uint32_t size = in_size[b];
        Rec*           R    = recs + rec_base[b];
        if (threadIdx.x == 0)
        {
            sh_i = 0;
            sh_dst = 0;
            sh_n = 0;
            sh_err = 0;
        }
        __syncthreads();
        while (true)
        {
            const uint32_t w0 = sh_i;
            if (w0 >= size || sh_err)
                break;
            const uint32_t wl = min(WIN, size - w0);
            for (uint32_t k = threadIdx.x; k < wl; k += 64)
                win[k] = src[w0 + k];
            __syncthreads();
            if (threadIdx.x == 0)
            {
                uint32_t i = w0, dst = sh_dst, n = sh_n;
                while (i < size && i < w0 + wl)
                {
                    const int c = (int8_t) win[i - w0];
                    if (c >= 0)
                    {
                        if (i + 1 + (uint32_t) c + 1 > size)
                        {
                            sh_err = 1;
                            break;
                        }
                        R[n++] = Rec{i, dst};
                        dst += (uint32_t) c + 1;
                        i += (uint32_t) c + 2;
                    }
                    else if (c >= -127)
                    {
                        if (i + 1 >= size)
                        {
                            sh_err = 1;
                            break;
                        }
                        R[n++] = Rec{i, dst};
                        dst += (uint32_t) (1 - c);
                        i += 2;
                    }
                    else
                        i += 1;
                }
                sh_i   = i;
                sh_dst = dst;
                sh_n   = n;
            }
            __syncthreads();
        }
        if (threadIdx.x == 0)
        {
            nrec[b]     = sh_n;
            out_size[b] = sh_err ? 0 : sh_dst;
        }
        __syncthreads();
    }
}

// expand records: grid.y = block
__global__ void k_rled_expand(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_base, uint32_t nblocks,
                              const Rec* __restrict__ recs, const uint64_t* __restrict__ rec_base, const uint32_t* __restrict__ nrec,
                              const uint32_t* __restrict__ out_size, uint8_t* __restrict__ out, const uint64_t* __restrict__ out_base,
                              const uint64_t* __restrict__ out_cap)
{
    for (uint32_t b = blockIdx.y; b < nblocks; b += gridDim.y)
    {
        const uint32_t os = out_size[b];
        if (os == 0 || os > out_cap[b])
            continue;
        const uint8_t* src = in + in_base[b];
        const Rec*     R   = recs + rec_base[b];
        uint8_t*       dst = out + out_base[b];
        const uint32_t n   = nrec[b];
        for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x)
        {
            const Rec E = R[r];
            const int c = (int8_t) src[E.src];
            if (c >= 0)
                for (int k = 0; k <= c; ++k)
                    dst[E.dst + k] = src[E.src + 1 + k];
            else
            {
                const uint8_t v = src[E.src + 1];
                for (int k = 0; k < 1 - c; ++k)
                    dst[E.dst + k] = v;
            }
        }
    }
}

}  // namespace

bool rle_decode_device(const uint8_t* d_in, const uint64_t* d_in_base, const uint32_t* d_in_size, uint32_t nblocks, uint8_t* d_out,
                       const uint64_t* d_out_base, const uint64_t* d_out_cap, uint32_t* d_out_size, void* d_recs, const uint64_t* d_rec_base,
                       uint32_t* d_nrec, hipStream_t s)
{
    Rec* recs = static_cast<Rec*>(d_recs);
    hipLaunchKernelGGL(k_rled_parse, dim3(std::min<uint32_t>(nblocks, 65535)), dim3(64), 0, s, d_in, d_in_base, d_in_size, nblocks, recs,
                       d_rec_base, d_nrec, d_out_size);
    hipLaunchKernelGGL(k_rled_expand, dim3(64, std::min<uint32_t>(nblocks, 65535)), dim3(256), 0, s, d_in, d_in_base, nblocks, recs,
                       d_rec_base, d_nrec, d_out_size, d_out, d_out_base, d_out_cap);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace bra
