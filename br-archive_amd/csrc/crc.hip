// crc.hip -- CRC32C of the .BRa chunk stream and the chunk framing on the device.
//
// The reference folds a CRC32C over every chunk of a compressed file in its chunk loop
// (src/io/lib_bra_io_file_chunks.c:214,248-249): per chunk the 268-byte in-memory header, then the
// source chunk (combined in with bra_crc32c_combine, src/utils/lib_bra_crc32c.c:181-231).  That is
// the CRC32C of the virtual stream hdr0 || chunk0 || hdr1 || chunk1 || ...; the decode loop
// (:396-397) folds the same stream over the decoded bytes.  Here the stream is cut into 64 KiB
// pieces, one workgroup each, and every piece's contribution is moved to the end of the stream
// with GF(2) arithmetic, so the pieces are independent and their contributions simply XOR:
//
//   L(X)       = the raw CRC of X (zero initial register, no final complement); L is linear.
//   L(A || B)  = L(A) * x^(8|B|) ^ L(B)                     (mod P, reflected representation)
//   crc(X, prev) = ~((~prev) * x^(8|X|) ^ L(X))              (bra_crc32c, lib_bra_crc32c.c:102-117)
//
// Inside a workgroup thread t owns the 16-byte units t, t+256, ... of its piece (coalesced 16-byte
// loads); a unit's raw CRC is 16 independent LDS table lookups (slicing by 16), the running value
// moves one 4 KiB stride with 4 more lookups, and one multiplication by x^(8*16*(255-t)) lines the
// thread up with the piece end.  The piece value is then multiplied by x^(8*distance to the stream
// end) -- a product of at most 61 precomputed powers x^(2^k), formed as a wave-wide tree -- and
// XORed into the result word, which starts as the complement of (~prev) * x^(8|stream|).
//
// The constants (tables, powers) are generated at compile time from the polynomial.
#include "crc.h"

#include <algorithm>

namespace bra {
namespace {

constexpr uint32_t POLY   = 0x82F63B78u;  // reflected Castagnoli (lib_bra_crc32c.c:27)
constexpr uint32_t ONE    = 0x80000000u;  // x^0 in the reflected representation
constexpr int      CRC_TPB = 256;
constexpr int      UNITS  = 16;                       // units per thread per piece
constexpr uint32_t PIECE  = CRC_TPB * UNITS * 16;     // 64 KiB per workgroup
constexpr int      HDR_UNITS = (CHUNK_HDR_MEM + 15) / 16;  // 17 units per header, aligned to its end

__host__ __device__ constexpr uint32_t mulmod(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int k = 31; k >= 0; --k)
    {
        if ((a >> k) & 1u)
            p ^= b;
        b = (b >> 1) ^ ((b & 1u) ? POLY : 0u);
    }
    return p;
}

struct CrcConst
{
    uint32_t T[16][256];  // T[k][v]: raw CRC of byte v followed by k zero bytes
    uint32_t S[4][256];   // S[m][v]: (v << 8m) * x^(8 * 4096) -- one thread stride
    uint32_t K[256];      // K[j] = x^(8 * 16 * j)
    uint32_t X2N[64];     // X2N[k] = x^(2^k)
};

constexpr CrcConst make_crc_const()
{
    CrcConst c{};
    for (uint32_t v = 0; v < 256; ++v)
    {
        uint32_t r = v;
        for (int k = 0; k < 8; ++k)
            r = (r & 1u) ? (r >> 1) ^ POLY : r >> 1;
        c.T[0][v] = r;
    }
    for (int k = 1; k < 16; ++k)
        for (uint32_t v = 0; v < 256; ++v)
            c.T[k][v] = (c.T[k - 1][v] >> 8) ^ c.T[0][c.T[k - 1][v] & 0xFFu];
    c.X2N[0] = ONE >> 1;
    for (int k = 1; k < 64; ++k)
        c.X2N[k] = mulmod(c.X2N[k - 1], c.X2N[k - 1]);
    static_assert(CRC_TPB * 16 == 4096, "S is the shift by one 4 KiB stride");
    for (int m = 0; m < 4; ++m)
        for (uint32_t v = 0; v < 256; ++v)
            c.S[m][v] = mulmod(v << (8 * m), c.X2N[15]);  // x^(8 * 4096) = x^(2^15)
    c.K[0] = ONE;
    for (int j = 1; j < 256; ++j)
        c.K[j] = mulmod(c.K[j - 1], c.X2N[7]);  // x^(8 * 16) = x^(2^7)
    return c;
}

__constant__ CrcConst c_crc = make_crc_const();
constexpr CrcConst    h_crc = make_crc_const();

// x^(8n) for a wave-uniform n: lane k contributes x^(2^(k+3)) when bit k of n is set, then a
// 6-level product tree over the wave.  Every lane of the wave must call it; all get the result.
__device__ uint32_t wave_x8n(uint64_t n)
{
    const int lane = lane_id();
    uint32_t  f    = (lane < 61 && ((n >> lane) & 1u)) ? c_crc.X2N[lane + 3] : ONE;
#pragma unroll
    for (int m = 1; m < WAVE; m <<= 1)
        f = mulmod(f, (uint32_t) __shfl_xor((int) f, m, WAVE));
    return f;
}

__device__ __forceinline__ uint32_t sel4(uint32_t k, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    return k == 0 ? a : k == 1 ? b : k == 2 ? c : d;
}

// The 16 bytes at p (any alignment); bytes below `lo` read as zero (leading zeros do not change a
// raw CRC).  Requires p + 16 > lo; only aligned 16-byte words holding at least one byte of
// [lo, p + 16) are read.
__device__ __forceinline__ uint4 load16(const uint8_t* p, const uint8_t* lo)
{
    const uintptr_t a   = (uintptr_t) p;
    const uintptr_t a0  = a & ~(uintptr_t) 15;
    const uint32_t  mis = (uint32_t) (a & 15);
    const uint4     z   = make_uint4(0, 0, 0, 0);
    uint4           q0  = (a0 + 16 > (uintptr_t) lo) ? *reinterpret_cast<const uint4*>(a0) : z;
    uint4           r   = q0;
    if (mis)
    {
        const uint4    q1 = *reinterpret_cast<const uint4*>(a0 + 16);
        const uint32_t d[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const uint32_t w = mis >> 2, sh = mis & 3;
        uint32_t       e[5];
#pragma unroll
        for (int j = 0; j < 5; ++j)
            e[j] = sel4(w, d[j], d[j + 1], d[j + 2], d[j + 3]);
        r = make_uint4(__builtin_amdgcn_alignbyte(e[1], e[0], sh), __builtin_amdgcn_alignbyte(e[2], e[1], sh),
                       __builtin_amdgcn_alignbyte(e[3], e[2], sh), __builtin_amdgcn_alignbyte(e[4], e[3], sh));
    }
    if (a < (uintptr_t) lo)
    {
        const int nz    = (int) ((uintptr_t) lo - a);  // 1..15 leading bytes to clear
        uint32_t  v[4]  = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
        {
            const int c = nz - 4 * k;
            v[k]        = c >= 4 ? 0u : c <= 0 ? v[k] : v[k] & (0xFFFFFFFFu << (8 * c));
        }
        r = make_uint4(v[0], v[1], v[2], v[3]);
    }
    return r;
}

// Raw CRC of 16 bytes (byte i of the unit is followed by 15 - i more bytes).
__device__ __forceinline__ uint32_t crc16(const uint4 q, const uint32_t (*T)[256])
{
    const uint32_t v[4] = {q.x, q.y, q.z, q.w};
    uint32_t       r    = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            r ^= T[15 - (4 * d + j)][(v[d] >> (8 * j)) & 0xFFu];
    return r;
}

__device__ __forceinline__ uint32_t shift_stride(uint32_t c, const uint32_t (*S)[256])
{
    return S[0][c & 0xFFu] ^ S[1][(c >> 8) & 0xFFu] ^ S[2][(c >> 16) & 0xFFu] ^ S[3][c >> 24];
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
#pragma unroll
    for (int m = 1; m < WAVE; m <<= 1)
        v ^= (uint32_t) __shfl_xor((int) v, m, WAVE);
    return v;
}

struct StreamArgs
{
    const uint8_t* data;
    uint64_t       total;
    const uint8_t* hdr;   // nullptr: no headers
    uint64_t       V;     // stream length: total + nb * hb
    uint32_t       cs;    // chunk size
    uint32_t       hb;    // header bytes per chunk (268 or 0)
    uint32_t       nb;    // chunks
    uint32_t       ppc;   // pieces per chunk
    uint32_t*      crc;
    uint64_t       g0;    // global index of local chunk 0 in the (possibly sharded) stream
    uint64_t       gs;    // global index stride between local chunks (1 = contiguous)
};

// Workgroups [0, nb * ppc) take one 64 KiB piece of chunk data each (pieces aligned to the chunk
// end, the first one ragged); the workgroups after them take 4 chunk headers each (one per wave).
__global__ __launch_bounds__(CRC_TPB) void k_crc_stream(StreamArgs a, uint32_t n_pieces, uint32_t n_work)
{
    __shared__ uint32_t T[16][256];
    __shared__ uint32_t S[4][256];
    __shared__ uint32_t red[CRC_TPB / WAVE];
    for (uint32_t i = threadIdx.x; i < 16 * 256; i += CRC_TPB)
        (&T[0][0])[i] = (&c_crc.T[0][0])[i];
    for (uint32_t i = threadIdx.x; i < 4 * 256; i += CRC_TPB)
        (&S[0][0])[i] = (&c_crc.S[0][0])[i];
    __syncthreads();
    const uint32_t t = threadIdx.x, wv = t / WAVE, lane = t % WAVE;
    for (uint32_t w = blockIdx.x; w < n_work; w += gridDim.x)
    {
        if (w < n_pieces)
        {
            const uint32_t b     = w / a.ppc;
            const uint32_t prev  = a.ppc - 1 - w % a.ppc;  // pieces after this one in the chunk
            const uint64_t c0    = (uint64_t) b * a.cs;
            const uint32_t s     = (uint32_t) min<uint64_t>(a.cs, a.total - c0);
            const int64_t  pend  = (int64_t) s - (int64_t) prev * PIECE;  // chunk-local piece end
            if (pend <= 0)
                continue;  // uniform: ragged last chunk has fewer pieces
            const uint8_t* chunk = a.data + c0;
            const uint8_t* lo    = chunk + max<int64_t>(0, pend - (int64_t) PIECE);
            uint32_t       acc   = 0;
#pragma unroll 4
            for (int i = 0; i < UNITS; ++i)
            {
                const int64_t u = pend - (int64_t) PIECE + 16 * (int64_t) (t + CRC_TPB * i);
                acc             = shift_stride(acc, S);
                if (u + 16 > 0)
                    acc ^= crc16(load16(chunk + u, lo), T);
            }
            acc = mulmod(acc, c_crc.K[CRC_TPB - 1 - t]);
            acc = wave_xor(acc);
            if (lane == 0)
                red[wv] = acc;
            __syncthreads();
            if (wv == 0)
            {
                uint32_t v = 0;
#pragma unroll
                for (int k = 0; k < CRC_TPB / WAVE; ++k)
                    v ^= red[k];
                const uint64_t g   = a.g0 + (uint64_t) b * a.gs;  // global chunk index
                const uint64_t end = g * (a.cs + a.hb) + a.hb + (uint64_t) pend;  // stream position
                const uint32_t f   = wave_x8n(a.V - end);
                if (lane == 0)
                    atomicXor(a.crc, mulmod(v, f));
            }
            __syncthreads();
        }
        else
        {
            // headers: wave wv handles chunk header b; lane j < 17 one unit aligned to the header end
            const uint32_t b = (w - n_pieces) * (CRC_TPB / WAVE) + wv;
            if (b >= a.nb)
                continue;  // wave-uniform; no block barrier on this path
            const uint8_t* h   = a.hdr + (uint64_t) b * CHUNK_HDR_MEM;
            uint32_t       acc = 0;
            if (lane < HDR_UNITS)
            {
                const int u = (int) CHUNK_HDR_MEM - 16 * (HDR_UNITS - (int) lane);  // -4, 12, ..., 252
                acc         = mulmod(crc16(load16(h + u, h), T), c_crc.K[HDR_UNITS - 1 - lane]);
            }
            acc                = wave_xor(acc);
            const uint64_t end = (a.g0 + (uint64_t) b * a.gs) * (a.cs + a.hb) + a.hb;
            const uint32_t f   = wave_x8n(a.V - end);
            if (lane == 0)
                atomicXor(a.crc, mulmod(acc, f));
        }
    }
}

// ---- framing ------------------------------------------------------------------------------------

// dst[0, n) = src[0, n): aligned 16-byte stores in the middle, byte stores at the two edges (so
// neighbouring records written by other workgroups are never touched).
__device__ void copy_bytes(uint8_t* dst, const uint8_t* src, uint64_t n)
{
    const uint64_t head = min<uint64_t>(n, (16 - ((uintptr_t) dst & 15)) & 15);
    for (uint64_t i = threadIdx.x; i < head; i += blockDim.x)
        dst[i] = src[i];
    const uint64_t nw   = (n - head) / 16;
    const uint64_t tail = head + 16 * nw;
    uint4*         d4   = reinterpret_cast<uint4*>(dst + head);
    const uint8_t* s    = src + head;
    for (uint64_t k = threadIdx.x; k < nw; k += blockDim.x)
        d4[k] = load16(s + 16 * k, s);
    for (uint64_t i = tail + threadIdx.x; i < n; i += blockDim.x)
        dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_frame(const uint8_t* __restrict__ hdr, const uint64_t* __restrict__ poff,
                                               const uint8_t* __restrict__ pay, uint32_t nb, uint8_t* __restrict__ out)
{
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x)
    {
        const uint64_t p0  = poff[b], esz = poff[b + 1] - p0;
        uint8_t*       rec = out + p0 + (uint64_t) CHUNK_HDR_DISK * b;
        const uint8_t* h   = hdr + (uint64_t) CHUNK_HDR_MEM * b;
        for (uint32_t i = threadIdx.x; i < CHUNK_HDR_DISK; i += blockDim.x)
            rec[i] = h[i < 3 ? i : i + 1];  // 3 low bytes of pi, then the packed bra_huffman_t
        copy_bytes(rec + CHUNK_HDR_DISK, pay + p0, esz);
    }
}

__device__ __forceinline__ uint32_t rd32(const uint8_t* p)
{
    return (uint32_t) p[0] | ((uint32_t) p[1] << 8) | ((uint32_t) p[2] << 16) | ((uint32_t) p[3] << 24);
}

// One thread follows the record chain (each record's length is in its own header).
__global__ void k_unframe_walk(const uint8_t* __restrict__ st, uint64_t size, uint32_t cap, uint64_t* __restrict__ poff,
                               uint32_t* __restrict__ status)
{
    if (threadIdx.x != 0 || blockIdx.x != 0)
        return;
    uint64_t pos = 0;
    uint32_t n = 0, err = 0;
    while (pos < size)
    {
        if (n >= cap || size - pos < CHUNK_HDR_DISK)
        {
            err = 1;
            break;
        }
        const uint32_t esz = rd32(st + pos + 3 + 260);
        poff[n++]          = pos + CHUNK_HDR_DISK;
        if (esz > size - pos - CHUNK_HDR_DISK)
        {
            err = 1;
            break;
        }
        pos += CHUNK_HDR_DISK + esz;
    }
    status[0] = n;
    status[1] = err;
}

// Rebuild the 268-byte in-memory headers and validate them (lib_bra_io_file_chunks.c:31-49).
__global__ __launch_bounds__(256) void k_unframe_headers(const uint8_t* __restrict__ st, const uint64_t* __restrict__ poff,
                                                         uint32_t cap, uint32_t max_chunk, uint8_t* __restrict__ hdr,
                                                         uint32_t* __restrict__ status)
{
    const uint32_t n = min(status[0], cap);
    for (uint32_t b = blockIdx.x; b < n; b += gridDim.x)
    {
        const uint8_t* r = st + poff[b] - CHUNK_HDR_DISK;
        uint8_t*       h = hdr + (uint64_t) CHUNK_HDR_MEM * b;
        for (uint32_t i = threadIdx.x; i < CHUNK_HDR_MEM; i += blockDim.x)
            h[i] = i < 3 ? r[i] : i == 3 ? 0 : r[i - 1];
        if (threadIdx.x == 0)
        {
            const uint32_t pi = (uint32_t) r[0] | ((uint32_t) r[1] << 8) | ((uint32_t) r[2] << 16);
            const uint32_t os = rd32(r + 3 + 256), es = rd32(r + 3 + 260);
            if (pi >= max_chunk || es > max_chunk || os > max_chunk || es == 0 || os == 0)
                atomicOr(status + 1, 2u);
        }
    }
}

// ---- assembly of sharded encoder output ---------------------------------------------------------

// Source of global block g: part g % P at local index g / P (round robin), or the part whose
// contiguous range holds g.
__device__ __forceinline__ void shard_src(const ShardParts& P, uint32_t g, uint32_t& part, uint32_t& loc)
{
    if (P.round_robin)
    {
        part = g % P.n;
        loc  = g / P.n;
        return;
    }
    part = 0;
    while (part + 1 < P.n && g >= P.first[part + 1])
        ++part;
    loc = g - P.first[part];
}

__device__ __forceinline__ uint32_t hdr_encoded_size(const uint8_t* h) { return rd32(h + CHUNK_HDR_MEM - 4); }

// One workgroup: exclusive scan of the encoded sizes in global block order -> out offsets
// (nb + 1 entries; the last one is the total payload, or UINT64_MAX when it exceeds cap: then the
// last block is not copied and the caller sees the overflow without a host round trip).
__global__ __launch_bounds__(1024) void k_shard_offsets(ShardParts P, uint32_t nb, uint64_t* __restrict__ off_out, uint64_t cap,
                                                        uint64_t* __restrict__ need)
{
    __shared__ uint64_t part_sum[1024 / WAVE];
    __shared__ uint64_t carry_s;
    if (threadIdx.x == 0)
        carry_s = 0;
    __syncthreads();
    const int lane = lane_id(), w = threadIdx.x / WAVE;
    for (uint32_t c0 = 0; c0 < nb; c0 += 1024)
    {
        const uint32_t g = c0 + threadIdx.x;
        uint64_t       v = 0;
        if (g < nb)
        {
            uint32_t part, loc;
            shard_src(P, g, part, loc);
            v = hdr_encoded_size(P.hdr[part] + (uint64_t) CHUNK_HDR_MEM * loc);
        }
        uint64_t x = v;  // inclusive wave scan
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1)
        {
            const uint64_t y = shfl_up64(x, d);
            if (lane >= d)
                x += y;
        }
        if (lane == WAVE - 1)
            part_sum[w] = x;
        __syncthreads();
        uint64_t before = carry_s, all = 0;
        for (int k = 0; k < 1024 / WAVE; ++k)
        {
            if (k < w)
                before += part_sum[k];
            all += part_sum[k];
        }
        if (g < nb)
            off_out[g] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 0)
            carry_s += all;
        __syncthreads();
    }
    if (threadIdx.x == 0)
    {
        off_out[nb] = carry_s > cap ? ~0ull : carry_s;
        *need       = carry_s;  // the payload size the assembly needs, also on overflow
    }
}

// One workgroup per global block: its 268-byte header and payload into global order.  A block that
// would end past `cap` is not written and sets *err.
__global__ __launch_bounds__(256) void k_shard_copy(ShardParts P, uint32_t nb, const uint64_t* __restrict__ off_out, uint8_t* __restrict__ hdr_out,
                                                    uint8_t* __restrict__ pay_out, uint64_t cap, uint32_t* __restrict__ err)
{
    for (uint32_t g = blockIdx.x; g < nb; g += gridDim.x)
    {
        uint32_t part, loc;
        shard_src(P, g, part, loc);
        const uint8_t* h = P.hdr[part] + (uint64_t) CHUNK_HDR_MEM * loc;
        for (uint32_t i = threadIdx.x; i < CHUNK_HDR_MEM; i += blockDim.x)
            hdr_out[(uint64_t) CHUNK_HDR_MEM * g + i] = h[i];
        const uint64_t o = off_out[g], esz = off_out[g + 1] - o;
        if (o + esz > cap)
        {
            if (threadIdx.x == 0)
                atomicOr(err, 1u);
            continue;
        }
        copy_bytes(pay_out + o, P.pay[part] + P.off[part][loc], esz);
    }
}

}  // namespace

uint32_t crc_mulmod(uint32_t a, uint32_t b) { return mulmod(a, b); }

uint32_t crc_x8n(uint64_t n)
{
    uint32_t p = ONE;
    for (int k = 3; n && k < 64; ++k, n >>= 1)
        if (n & 1)
            p = mulmod(p, h_crc.X2N[k]);
    return p;
}

uint32_t crc32c_host(const void* data, uint64_t len, uint32_t prev)
{
    const uint8_t* p = static_cast<const uint8_t*>(data);
    uint32_t       c = ~prev;
    for (uint64_t i = 0; i < len; ++i)
        c = h_crc.T[0][(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    return ~c;
}

uint32_t crc32c_combine_host(uint32_t a, uint32_t b, uint64_t len_b) { return len_b ? mulmod(a, crc_x8n(len_b)) ^ b : a; }

bool crc_stream_shard_device(const uint8_t* d_data, uint64_t total, uint32_t chunk_size, const uint8_t* d_hdr, uint64_t g0, uint64_t gstride,
                             uint64_t global_total, uint32_t prev, bool with_init, uint32_t* d_crc, hipStream_t s)
{
    if (!d_crc || (total && !d_data) || gstride == 0 || total > global_total)
        return false;
    StreamArgs a{};
    a.data  = d_data;
    a.total = total;
    a.hdr   = d_hdr;
    a.hb    = d_hdr ? CHUNK_HDR_MEM : 0;
    a.cs    = d_hdr ? chunk_size : (1u << 30);
    if (a.cs == 0 || (!d_hdr && (g0 != 0 || gstride != 1 || total != global_total)))
        return false;
    a.nb  = (uint32_t) ((total + a.cs - 1) / a.cs);
    a.ppc = (a.cs + PIECE - 1) / PIECE;
    a.g0  = g0;
    a.gs  = gstride;
    const uint64_t nbg = (global_total + a.cs - 1) / a.cs;
    if (a.nb && g0 + (uint64_t) (a.nb - 1) * gstride >= nbg)
        return false;
    if (a.nb)
    {
        // only the global last chunk may be ragged, and it must be this shard's last one
        const uint64_t gl    = g0 + (uint64_t) (a.nb - 1) * gstride;
        const uint64_t want  = std::min<uint64_t>(a.cs, global_total - gl * a.cs);
        const uint64_t local = total - (uint64_t) (a.nb - 1) * a.cs;
        if (want != local)
            return false;
    }
    a.V   = global_total + nbg * a.hb;
    a.crc = d_crc;
    // the result word starts as ~((~prev) * x^(8V)) in exactly one shard; every piece XORs in its raw
    // contribution moved to the end of the global stream, so the shards' words XOR to the stream CRC
    const uint32_t init = with_init ? ~mulmod(~prev, crc_x8n(a.V)) : 0u;
    BRA_HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_crc), (int) init, 1, s));
    const uint64_t n_pieces = (uint64_t) a.nb * a.ppc;
    const uint64_t n_hdr    = a.hb ? (a.nb + CRC_TPB / WAVE - 1) / (CRC_TPB / WAVE) : 0;
    const uint64_t n_work   = n_pieces + n_hdr;
    if (n_work == 0)
        return true;
    if (n_work >= (1ull << 31))
        return false;
    const uint32_t grid = (uint32_t) std::min<uint64_t>(n_work, 1u << 20);
    hipLaunchKernelGGL(k_crc_stream, dim3(grid), dim3(CRC_TPB), 0, s, a, (uint32_t) n_pieces, (uint32_t) n_work);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

bool crc_stream_device(const uint8_t* d_data, uint64_t total, uint32_t chunk_size, const uint8_t* d_hdr, uint32_t prev, uint32_t* d_crc,
                       hipStream_t s)
{
    return crc_stream_shard_device(d_data, total, chunk_size, d_hdr, 0, 1, total, prev, true, d_crc, s);
}

bool frame_chunks_device(const uint8_t* d_hdr, const uint64_t* d_payload_off, const uint8_t* d_payload, uint32_t nb, uint8_t* d_out,
                         hipStream_t s)
{
    if (nb == 0)
        return true;
    hipLaunchKernelGGL(k_frame, dim3(std::min<uint32_t>(nb, 65535)), dim3(256), 0, s, d_hdr, d_payload_off, d_payload, nb, d_out);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

bool unframe_chunks_device(const uint8_t* d_stream, uint64_t size, uint32_t cap, uint32_t max_chunk, uint8_t* d_hdr, uint64_t* d_payload_off,
                           uint32_t* d_status, hipStream_t s)
{
    hipLaunchKernelGGL(k_unframe_walk, dim3(1), dim3(64), 0, s, d_stream, size, cap, d_payload_off, d_status);
    BRA_HIP_CHECK(hipGetLastError());
    if (cap)
    {
        hipLaunchKernelGGL(k_unframe_headers, dim3(std::min<uint32_t>(cap, 65535)), dim3(256), 0, s, d_stream, d_payload_off, cap, max_chunk,
                           d_hdr, d_status);
        BRA_HIP_CHECK(hipGetLastError());
    }
    return true;
}

bool assemble_shards_device(const ShardParts& parts, uint32_t nb, uint8_t* d_hdr_out, uint64_t* d_off_out, uint8_t* d_pay_out, uint64_t cap,
                            uint32_t* d_err, uint64_t* d_need, hipStream_t s)
{
    if (parts.n == 0 || parts.n > MAX_SHARDS || nb == 0)
        return false;
    BRA_HIP_CHECK(hipMemsetAsync(d_err, 0, 4, s));
    hipLaunchKernelGGL(k_shard_offsets, dim3(1), dim3(1024), 0, s, parts, nb, d_off_out, cap, d_need);
    BRA_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_shard_copy, dim3(std::min<uint32_t>(nb, 65535)), dim3(256), 0, s, parts, nb, d_off_out, d_hdr_out, d_pay_out, cap, d_err);
    BRA_HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace bra
