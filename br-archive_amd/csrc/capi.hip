// capi.hip -- the C-ABI of libbra_hip.so (include/bra_hip.h): the reference's 14 encoder entry
// points (single block, host buffers) and the batched device-resident codec.
#include "../../include/bra_hip.h"

#include "bwt.h"
#include "crc.h"
#include "huffman.h"
#include "ibwt.h"
#include "mtf.h"
#include "rle.h"
#include "prof.h"

#include <cstdarg>
#include <cstring>
#include <mutex>
#include <vector>

extern "C" void bra_log_error(const char* fmt, ...) __attribute__((weak));

void bra_hip_report(const char* fmt, ...)
{
    char    buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (bra_log_error)
        bra_log_error("%s", buf);
    else
        fprintf(stderr, "[bra_hip] %s\n", buf);
}

static_assert(sizeof(bra_io_chunk_header_t) == 268, "in-memory chunk header layout (lib_bra_types.h:63-68)");
static_assert(sizeof(bra_huffman_t) == 264, "bra_huffman_t layout");
static_assert(offsetof(bra_huffman_chunk_t, data) == 264, "bra_huffman_chunk_t layout");

using namespace bra;

// ---- event profiler (prof.h) ----
namespace bra {
thread_local Prof* g_prof = nullptr;

const char* prof_name(int slot)
{
    static const char* names[P_NSLOT] = {
        "stage.bwt", "stage.mtf", "stage.rle", "stage.huffman",
        "bwt.l0_hist", "bwt.l0_scatter", "bwt.pack", "bwt.hist", "bwt.scan", "bwt.scatter", "bwt.jobs", "bwt.mjobs", "bwt.fallback",
        "mtf.lastocc", "mtf.scan", "mtf.encode",
        "rle.runs", "rle.link", "rle.sizes", "rle.offsets", "rle.write",
        "huf.build", "huf.offsets", "huf.tilebits", "huf.tilescan", "huf.zero", "huf.pack",
        "chunks.frame", "chunks.crc",
        "dec.huffman", "dec.rle", "dec.mtf", "dec.ibwt",
        "dec.hd_trans", "dec.rled", "dec.mtf_local", "dec.ib_walk", "dec.ib_pair"};
    return (slot >= 0 && slot < P_NSLOT) ? names[slot] : "";
}

hipEvent_t Prof::get()
{
    if (!pool.empty())
    {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void) hipEventCreate(&e);
    return e;
}

void Prof::collect()
{
    for (int i = 0; i < P_NSLOT; ++i)
    {
        for (auto& pr : pending[i])
        {
            float ms_ = 0.f;
            (void) hipEventSynchronize(pr.second);
            if (hipEventElapsedTime(&ms_, pr.first, pr.second) == hipSuccess)
            {
                ms[i] += ms_;
                launches[i] += 1;
            }
            pool.push_back(pr.first);
            pool.push_back(pr.second);
        }
        pending[i].clear();
    }
}

void Prof::reset()
{
    collect();
    for (int i = 0; i < P_NSLOT; ++i)
    {
        ms[i]       = 0;
        launches[i] = 0;
        bytes[i]    = 0;
    }
}

Prof::~Prof()
{
    collect();
    for (hipEvent_t e : pool)
        (void) hipEventDestroy(e);
}
}  // namespace bra

namespace {

__global__ void k_headers(const uint32_t* __restrict__ pi, const HuffMetaRec* __restrict__ meta, uint32_t nb,
                          bra_io_chunk_header_t* __restrict__ hdr)
{
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x)
    {
        uint8_t*       dst = reinterpret_cast<uint8_t*>(hdr + b);
        const uint8_t* src = reinterpret_cast<const uint8_t*>(meta + b);
        for (uint32_t i = threadIdx.x; i < 268; i += blockDim.x)
            dst[i] = (i < 4) ? (uint8_t) (pi[b] >> (8 * i)) : src[i - 4];
    }
}

__global__ void k_split_headers(const bra_io_chunk_header_t* __restrict__ hdr, uint32_t nb, uint32_t* __restrict__ pi,
                                HuffMetaRec* __restrict__ meta)
{
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x)
    {
        const uint8_t* src = reinterpret_cast<const uint8_t*>(hdr + b);
        uint8_t*       dst = reinterpret_cast<uint8_t*>(meta + b);
        for (uint32_t i = threadIdx.x; i < 264; i += blockDim.x)
            dst[i] = src[i + 4];
        if (threadIdx.x == 0)
            pi[b] = hdr[b].primary_index;
    }
}

// Grow p to at least `need` elements; cap is set only once the allocation succeeded (dev_alloc).
template <typename T>
bool grow(T*& p, uint64_t& cap, uint64_t need)
{
    if (need <= cap)
        return true;
    cap              = 0;
    const uint64_t c = need + need / 8 + 256;
    if (!dev_alloc(p, c))
        return false;
    cap = c;
    return true;
}

// Makes `dev` current for the scope of a C-ABI call and restores the caller's device afterwards, so
// a call never silently changes the calling thread's current HIP device.
struct DevGuard
{
    int  prev = -1;
    bool ok   = false;
    explicit DevGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        ok = prev == dev || hipSetDevice(dev) == hipSuccess;
    }
    ~DevGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev)
            (void) hipSetDevice(prev);
    }
    DevGuard(const DevGuard&)            = delete;
    DevGuard& operator=(const DevGuard&) = delete;
};

}  // namespace

struct bra_gpu_ctx_s
{
    int            device = 0;
    hipStream_t    stream = nullptr;
    BwtWorkspace*  bwt    = nullptr;
    MtfWorkspace   mtf;
    RleWorkspace   rle;
    HuffWorkspace  huf;
    IbwtWorkspace  ib;
    Tiling         hist_tiling;
    // batch buffers
    uint8_t*       d_L = nullptr;
    uint8_t*       d_mtf = nullptr;
    uint8_t*       d_rle = nullptr;
    uint8_t*       d_tmp = nullptr;
    uint64_t       cap_L = 0, cap_mtf = 0, cap_rle = 0, cap_tmp = 0;
    BlockDesc*     d_blocks = nullptr;
    uint32_t*      d_pi = nullptr;
    uint32_t*      d_rle_size = nullptr;
    uint32_t*      d_hist = nullptr;
    uint32_t*      d_status = nullptr;
    uint64_t*      d_rle_base = nullptr;
    uint64_t*      d_rle_cap = nullptr;
    uint64_t*      d_aux = nullptr;  // block offsets for decode, record bases
    HuffMetaRec*   d_meta = nullptr;
    uint64_t       cap_b = 0, cap_pi = 0, cap_rs = 0, cap_hist = 0, cap_st = 0, cap_rb = 0, cap_rc = 0, cap_aux = 0, cap_meta = 0;
    // single-call staging
    uint8_t*       d_io = nullptr;
    uint64_t       cap_io = 0;
    uint64_t*      d_off = nullptr;
    uint64_t       cap_off = 0;
    uint8_t*       d_pay = nullptr;
    uint64_t       cap_pay = 0;
    bra_io_chunk_header_t* d_hdr = nullptr;
    uint64_t       cap_hdr = 0;
    uint32_t       last_nblocks = 0;
    uint32_t*      d_word = nullptr;  // [0] CRC result, [1..2] unframe status
    uint64_t       cap_word = 0;
    // encode geometry cache (encode_impl)
    std::vector<BlockDesc> enc_geo;
    BlockDesc*     d_enc_blocks = nullptr;
    uint8_t*       d_hin = nullptr;   // host-buffer chunk loops: staged input / output
    uint8_t*       d_hout = nullptr;
    uint64_t       cap_hin = 0, cap_hout = 0;
    uint64_t*      d_enc_rle_base = nullptr;
    uint64_t       cap_eb = 0, cap_erb = 0;
    hipEvent_t     null_ev = nullptr;  // CallStream: the null stream's position at a NULL-stream call
    hipEvent_t     caller_ev = nullptr;  // CallStream: the end of the last call on a caller-supplied stream
    bool           caller_pending = false;
    Prof           prof;
    // pipelined host-buffer chunk compression (bra_gpu_compress_chunks_submit / _collect)
    struct PipeSlot
    {
        uint8_t*   d_in = nullptr;
        uint8_t*   d_out = nullptr;
        uint64_t   cap_in = 0, cap_out = 0;
        hipEvent_t ev_in = nullptr, ev_done = nullptr;
        uint64_t   data_size = 0;
        uint32_t   nb = 0;
        int        state = 0;  // 0 free, 1 submitted
        // an input copy queued ahead by bra_gpu_compress_chunks_stage (the slot's next batch)
        bool           staged = false;
        const uint8_t* st_ptr = nullptr;
        uint64_t       st_size = 0;
    } pipe[2];
    hipStream_t    copy_in = nullptr, copy_out = nullptr;
    uint64_t*      h_pipe_mail = nullptr;  // pinned: per slot {payload bytes, chunk-stream CRC}
};

static bool ctx_init(bra_gpu_ctx_s* c, int device)
{
    c->device = device;
    DevGuard dg(device);
    if (!dg.ok)
        return false;
    BRA_HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    BRA_HIP_CHECK(hipEventCreateWithFlags(&c->null_ev, hipEventDisableTiming));
    c->bwt = bwt_workspace_create();
    return c->bwt != nullptr;
}

static void ctx_free(bra_gpu_ctx_s* c)
{
    DevGuard dg(c->device);
    bwt_workspace_destroy(c->bwt);
    c->mtf.release();
    c->rle.release();
    c->huf.release();
    c->ib.release();
    c->hist_tiling.release();
    void* ptrs[] = {c->d_L,       c->d_mtf,   c->d_rle,  c->d_tmp,  c->d_blocks, c->d_pi,  c->d_rle_size, c->d_hist, c->d_status, c->d_rle_base,
                    c->d_rle_cap, c->d_aux,   c->d_meta, c->d_io,     c->d_off, c->d_pay,      c->d_hdr,
                    c->d_word,    c->d_enc_blocks, c->d_enc_rle_base, c->d_hin, c->d_hout};
    for (void* p : ptrs)
        (void) hipFree(p);
    for (auto& ps : c->pipe)
    {
        (void) hipFree(ps.d_in);
        (void) hipFree(ps.d_out);
        if (ps.ev_in)
            (void) hipEventDestroy(ps.ev_in);
        if (ps.ev_done)
            (void) hipEventDestroy(ps.ev_done);
    }
    if (c->h_pipe_mail)
        (void) hipHostFree(c->h_pipe_mail);
    if (c->copy_in)
        (void) hipStreamDestroy(c->copy_in);
    if (c->copy_out)
        (void) hipStreamDestroy(c->copy_out);
    if (c->stream)
        (void) hipStreamDestroy(c->stream);
    if (c->null_ev)
        (void) hipEventDestroy(c->null_ev);
    if (c->caller_ev)
        (void) hipEventDestroy(c->caller_ev);
}

// The stream a batch call runs on (include/bra_hip.h, Part 2/3).  An explicit stream orders the
// call on that stream.  NULL means the context's stream, started after the work already queued on
// the null (legacy default) stream -- the caller's preceding copies, and torch's default stream,
// whose handle is NULL -- and complete when the call returns.  (The context stream is
// non-blocking: without the two joins a NULL-stream caller could read the results before the
// call's last kernels had written them -- the encode chain queues MTF / RLE / Huffman after its
// last host wait -- or the call could read inputs still in flight on the null stream.)
// A pipelined batch (bra_gpu_compress_chunks_submit) leaves its MTF / RLE / Huffman, framing and
// CRC queued on the context stream, and they use the context-wide work buffers; a call on a
// caller-supplied stream made before that batch is collected waits for the batch's end (the slot's
// ev_done), and the next submit waits for the last caller-stream call (caller_ev), so the two never
// share the buffers at the same time.
struct CallStream
{
    bra_gpu_ctx_s* c;
    hipStream_t    s;
    bool           own;
    CallStream(bra_gpu_ctx_s* ctx, void* stream) : c(ctx), s(stream ? (hipStream_t) stream : ctx->stream), own(stream == nullptr)
    {
        if (own && hipEventRecord(c->null_ev, nullptr) == hipSuccess)
            (void) hipStreamWaitEvent(s, c->null_ev, 0);
        if (!own)
            for (auto& ps : c->pipe)
                if (ps.state == 1)
                    (void) hipStreamWaitEvent(s, ps.ev_done, 0);
    }
    void mark()
    {
        if (own || (!c->caller_ev && hipEventCreateWithFlags(&c->caller_ev, hipEventDisableTiming) != hipSuccess))
            return;
        if (hipEventRecord(c->caller_ev, s) == hipSuccess)
            c->caller_pending = true;
    }
    // The call's result folded with the completion of a NULL-stream call: a kernel of the chain
    // that failed after the last host wait shows only at this synchronisation.
    int finish(int rc)
    {
        mark();
        if (own)
        {
            own = false;
            if (hipStreamSynchronize(s) != hipSuccess && rc >= 0)
                rc = -1;
        }
        else
            s = nullptr;  // marked
        return rc;
    }
    ~CallStream()
    {
        if (own)  // an early (error) return: still leave nothing queued behind the caller
            (void) hipStreamSynchronize(s);
        else if (s)
            mark();
    }
    operator hipStream_t() const { return s; }
};

static std::vector<BlockDesc> geometry(uint64_t total, uint32_t block_size)
{
    std::vector<BlockDesc> v;
    for (uint64_t off = 0; off < total; off += block_size)
        v.push_back(BlockDesc{off, (uint32_t) std::min<uint64_t>(block_size, total - off), 0});
    return v;
}

static bool ensure_block_arrays(bra_gpu_ctx_s* c, uint32_t nb)
{
    return grow(c->d_blocks, c->cap_b, nb) && grow(c->d_pi, c->cap_pi, nb) && grow(c->d_rle_size, c->cap_rs, nb) &&
           grow(c->d_hist, c->cap_hist, (uint64_t) nb * 256) && grow(c->d_status, c->cap_st, nb) && grow(c->d_rle_base, c->cap_rb, nb + 1) &&
           grow(c->d_rle_cap, c->cap_rc, nb + 1) && grow(c->d_aux, c->cap_aux, 2ull * nb + 2) && grow(c->d_meta, c->cap_meta, nb);
}

// The whole encode chain for a batch already in HBM.
static int encode_impl(bra_gpu_ctx_s* c, const uint8_t* d_in, const std::vector<BlockDesc>& hb, bra_io_chunk_header_t* d_headers,
                       uint64_t* d_payload_off, uint8_t* d_payload, uint64_t payload_cap, hipStream_t s, uint64_t* needed)
{
    const uint32_t nb = (uint32_t) hb.size();
    if (nb == 0)
        return -1;
    const uint64_t N = hb.back().off + hb.back().len;
    std::vector<uint64_t> rle_base(nb + 1);
    std::vector<BlockDesc> rle_blocks(nb);
    uint64_t R = 0;
    for (uint32_t b = 0; b < nb; ++b)
    {
        rle_base[b]   = R;
        rle_blocks[b] = BlockDesc{R, (uint32_t) rle_capacity(hb[b].len), 0};
        R += rle_capacity(hb[b].len);
    }
    rle_base[nb] = R;
    if (!ensure_block_arrays(c, nb) || !grow(c->d_L, c->cap_L, N + 16) || !grow(c->d_mtf, c->cap_mtf, N + 16) || !grow(c->d_rle, c->cap_rle, R + 16))
        return -1;
    // the block descriptors and RLE bases depend only on the geometry: uploaded once per geometry
    // (a pageable-source copy stalls the host, and the benchmark encodes one geometry repeatedly)
    if (c->enc_geo.size() != nb || std::memcmp(c->enc_geo.data(), hb.data(), nb * sizeof(BlockDesc)) != 0)
    {
        c->enc_geo.clear();
        if (!grow(c->d_enc_blocks, c->cap_eb, nb) || !grow(c->d_enc_rle_base, c->cap_erb, nb + 1) ||
            hipMemcpyAsync(c->d_enc_blocks, hb.data(), nb * sizeof(BlockDesc), hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(c->d_enc_rle_base, rle_base.data(), (nb + 1) * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -1;
        c->enc_geo = hb;
    }
    // The BWT is queued without waiting for its jobs; MTF, RLE and Huffman follow on the stream at
    // once.  Only then does the host wait for the jobs' mailbox: blocks whose rotations stayed tied
    // (periodic, highly repetitive) go through the prefix-doubling fallback, which rewrites their
    // L and pi, and the later stages are queued again.  With a payload capacity above the Huffman
    // bound (RLE bytes + a word per block) the chain has no other host wait, so the device never
    // idles while the host catches up.
    const bool cap_ok = payload_cap >= R + 16ull * nb + 64;
    uint64_t   total  = 0;
    const auto later_stages = [&]() -> int {
        {
            BRA_PROF(P_STAGE_MTF, s);
            // the BWT's per-block presence masks are the alphabets of its output too
            if (!mtf_encode_device(c->mtf, c->d_L, c->d_mtf, hb.data(), nb, s, bwt_alpha_masks(c->bwt)))
                return -1;
        }
        {
            BRA_PROF(P_STAGE_RLE, s);
            if (!rle_encode_device(c->rle, c->d_mtf, hb.data(), nb, c->d_enc_rle_base, c->d_rle, c->d_rle_size, c->d_hist, s))
                return -1;
        }
        bool hok = false;
        {
            BRA_PROF(P_STAGE_HUF, s);
            hok = huff_encode_device(c->huf, c->d_rle, rle_blocks.data(), nb, c->d_hist, c->d_rle_size, c->d_meta, d_payload_off, d_payload,
                                     payload_cap, &total, s, cap_ok);
        }
        if (!hok)
        {
            if (needed)
                *needed = total;
            return total + 8 > payload_cap ? -2 : -1;
        }
        hipLaunchKernelGGL(k_headers, dim3(std::min<uint32_t>(nb, 65535)), dim3(256), 0, s, c->d_pi, c->d_meta, nb, d_headers);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    };
    bool fallback = false;
    {
        BRA_PROF(P_STAGE_BWT, s);
        if (!bwt_encode_enqueue(c->bwt, d_in, c->d_enc_blocks, hb.data(), nb, c->d_L, c->d_pi, s))
            return -1;
    }
    int rc = later_stages();
    // (the fallback, when it runs, is timed by its own slot: one stage scope per call keeps the
    // stage slots' per-launch averages per step)
    if (!bwt_encode_finish(c->bwt, d_in, c->d_enc_blocks, hb.data(), nb, c->d_L, c->d_pi, s, &fallback))
        return -1;
    if (fallback)
        rc = later_stages();  // L changed
    if (rc != 0)
        return rc;
    constexpr uint64_t SIZE_SLOTS = 1ull << P_RLE_WRITE | 1ull << P_HUF_BUILD | 1ull << P_HUF_TILEBITS | 1ull << P_HUF_TILESCAN | 1ull << P_HUF_ZERO |
                                    1ull << P_HUF_PACK | 1ull << P_HUF_OFFSETS;
    if (g_prof && (g_prof->mask & SIZE_SLOTS))
    {
        // sizes of the RLE outputs for the byte accounting of rle.write / huf.* (profiling those
        // slots only: the copy waits for the step)
        std::vector<uint32_t> rs(nb);
        if (hipMemcpyAsync(rs.data(), c->d_rle_size, nb * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(&total, d_payload_off + nb, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return -1;
        double Rt = 0;
        for (uint32_t v : rs)
            Rt += v;
        const double ntiles = (double) c->huf.tiling.n;
        prof_bytes(P_RLE_WRITE, (double) N + Rt + 48.0 * c->rle.tiling.n);
        prof_bytes(P_HUF_BUILD, 1024.0 * nb + 264.0 * nb);
        prof_bytes(P_HUF_TILEBITS, Rt + 4.0 * ntiles);
        prof_bytes(P_HUF_TILESCAN, 12.0 * ntiles);
        prof_bytes(P_HUF_ZERO, 20.0 * ntiles);
        prof_bytes(P_HUF_PACK, Rt + (double) total + 12.0 * ntiles);
        prof_bytes(P_HUF_OFFSETS, 16.0 * nb);
    }
    c->last_nblocks = nb;
    if (needed)
    {
        // the caller wants the payload size on the host (the chunk loop frames and sizes its output)
        if (hipMemcpyAsync(&total, d_payload_off + nb, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return -1;
        *needed = total;
    }
    return 0;
}

// The whole decode chain.  d_out receives the blocks of geometry hb.  With `flex` (a .BRa chunk
// stream, lib_bra_io_file_chunks.c:340-420) hb only gives capacities: every chunk may decode to
// any size up to its hb[b].len, the primary index is checked against the decoded size (:383-387)
// as the reference does, and the chunks land back to back in d_out (*out_size bytes, at most
// out_cap).
static int decode_impl(bra_gpu_ctx_s* c, const bra_io_chunk_header_t* d_headers, const uint64_t* d_payload_off, const uint8_t* d_payload,
                       const std::vector<BlockDesc>& hb, uint8_t* d_out, hipStream_t s, bool flex = false, uint64_t out_cap = 0,
                       uint64_t* out_size = nullptr, std::vector<uint32_t>* out_sizes = nullptr)
{
    bwt_forget_jobs(c->bwt);  // the job phase of the last encode is no longer re-runnable
    const uint32_t nb = (uint32_t) hb.size();
    if (nb == 0)
        return -1;
    const uint64_t N = hb.back().off + hb.back().len;
    if (!ensure_block_arrays(c, nb))
        return -1;
    std::vector<bra_io_chunk_header_t> hh(nb);
    if (hipMemcpyAsync(hh.data(), d_headers, nb * sizeof(bra_io_chunk_header_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    // RLE streams back to back; record arrays; MTF input at the block offsets
    std::vector<uint64_t> rbase(nb), outb(nb), outcap(nb);
    std::vector<uint32_t> rsz(nb);
    uint64_t R = 0;
    for (uint32_t b = 0; b < nb; ++b)
    {
        const uint32_t os = hh[b].huffman.orig_size;
        if (!flex && hh[b].primary_index >= hb[b].len)
        {
            bra_hip_report("invalid primary index (%u) for chunk size %u", hh[b].primary_index, hb[b].len);
            return -1;
        }
        rbase[b]  = R;
        rsz[b]    = os;
        outb[b]   = hb[b].off;
        outcap[b] = hb[b].len;
        R += (uint64_t) os + 16;
    }
    if (!grow(c->d_rle, c->cap_rle, R + 16) || !grow(c->d_L, c->cap_L, N + 16) ||
        !grow(c->d_mtf, c->cap_mtf, N + 16) || !grow(c->d_tmp, c->cap_tmp, N + 16))
        return -1;
    uint64_t* d_rbase  = c->d_rle_base;
    uint64_t* d_outcap = c->d_rle_cap;
    uint64_t* d_outb   = c->d_aux + nb + 1;
    if (hipMemcpyAsync(c->d_blocks, hb.data(), nb * sizeof(BlockDesc), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_rbase, rbase.data(), nb * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_outcap, outcap.data(), nb * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_outb, outb.data(), nb * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(c->d_rle_size, rsz.data(), nb * 4, hipMemcpyHostToDevice, s) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_split_headers, dim3(std::min<uint32_t>(nb, 65535)), dim3(256), 0, s, d_headers, nb, c->d_pi, c->d_meta);
    std::vector<uint32_t> esz(nb);
    for (uint32_t b = 0; b < nb; ++b)
        esz[b] = hh[b].huffman.encoded_size;
    {
        BRA_PROF(P_DEC_HUF, s);
        if (!huff_decode_device(c->huf, c->d_meta, esz.data(), nb, d_payload, d_payload_off, c->d_rle, d_rbase, c->d_status, s))
            return -1;
    }
    uint32_t* d_dec_size = c->d_hist;           // nb words
    {
        BRA_PROF(P_DEC_RLE, s);
        if (!rle_decode_device(c->rle, rsz.data(), c->d_rle, d_rbase, c->d_rle_size, nb, c->d_mtf, d_outb, d_outcap, d_dec_size, s))
            return -1;
    }
    if (g_prof)
    {
        // algorithmic bytes of the RLE decode: reads r, writes n
        uint64_t r = 0;
        for (uint32_t b = 0; b < nb; ++b)
            r += rsz[b];
        prof_bytes(P_DEC_RLED, (double) r + (double) N);
    }
    std::vector<uint32_t> st(nb), dsz(nb);
    if (hipMemcpyAsync(st.data(), c->d_status, nb * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(dsz.data(), d_dec_size, nb * 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return -1;
    for (uint32_t b = 0; b < nb; ++b)
    {
        if (st[b])
        {
            bra_hip_report("huffman decode error in block %u", b);
            return -1;
        }
        if (!flex && dsz[b] != hb[b].len)
        {
            bra_hip_report("RLE decode of block %u gave %u bytes, expected %u", b, dsz[b], hb[b].len);
            return -1;
        }
    }
    if (!flex)
    {
        {
            BRA_PROF(P_DEC_MTF, s);
            if (!mtf_decode_device(c->mtf, c->d_mtf, c->d_L, c->d_tmp, hb.data(), nb, s))
                return -1;
        }
        {
            BRA_PROF(P_DEC_IBWT, s);
            if (!ibwt_device(c->ib, c->d_L, c->d_pi, c->d_blocks, hb.data(), nb, d_out, s))
                return -1;
        }
        return hipStreamSynchronize(s) == hipSuccess ? 0 : -1;
    }
    // chunk stream: the decoded sizes define the geometry
    std::vector<BlockDesc> g = hb;
    uint64_t               total = 0;
    bool                   packed = true;
    for (uint32_t b = 0; b < nb; ++b)
    {
        if (dsz[b] == 0)
        {
            bra_hip_report("unable to decode RLE in chunk %u", b);
            return -1;
        }
        if (hh[b].primary_index >= dsz[b])
        {
            bra_hip_report("invalid primary index (%u) for chunk size %u", hh[b].primary_index, dsz[b]);
            return -1;
        }
        g[b].len = dsz[b];
        packed   = packed && g[b].off == total;
        total += dsz[b];
    }
    if (out_size)
        *out_size = total;
    if (out_sizes)
    {
        out_sizes->resize(nb);
        for (uint32_t b = 0; b < nb; ++b)
            (*out_sizes)[b] = g[b].len;
    }
    if (total > out_cap)
    {
        bra_hip_report("decoded chunk stream needs %llu bytes, output holds %llu", (unsigned long long) total, (unsigned long long) out_cap);
        return -2;
    }
    if (hipMemcpyAsync(c->d_blocks, g.data(), nb * sizeof(BlockDesc), hipMemcpyHostToDevice, s) != hipSuccess)
        return -1;
    if (!mtf_decode_device(c->mtf, c->d_mtf, c->d_L, c->d_tmp, g.data(), nb, s))
        return -1;
    // a short chunk before the last leaves a gap in the capacity layout: decode to scratch, then pack
    uint8_t* dst = packed ? d_out : c->d_tmp;
    if (!ibwt_device(c->ib, c->d_L, c->d_pi, c->d_blocks, g.data(), nb, dst, s))
        return -1;
    if (!packed)
    {
        uint64_t o = 0;
        for (uint32_t b = 0; b < nb; o += g[b].len, ++b)
            if (hipMemcpyAsync(d_out + o, c->d_tmp + g[b].off, g[b].len, hipMemcpyDeviceToDevice, s) != hipSuccess)
                return -1;
    }
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -1;
}

// =================================================================================================
// Part 2: batch API
// =================================================================================================
extern "C" {

bra_gpu_ctx_t* bra_gpu_ctx_create(int device)
{
    if (device < 0 && hipGetDevice(&device) != hipSuccess)  // -1: the calling thread's current device
        return nullptr;
    auto* c = new bra_gpu_ctx_s();
    if (!ctx_init(c, device))
    {
        ctx_free(c);
        delete c;
        return nullptr;
    }
    return c;
}

void bra_gpu_ctx_destroy(bra_gpu_ctx_t* c)
{
    if (!c)
        return;
    ctx_free(c);
    delete c;
}

uint32_t bra_gpu_num_blocks(uint64_t total, uint32_t block_size) { return block_size ? (uint32_t) ((total + block_size - 1) / block_size) : 0; }

uint64_t bra_gpu_payload_bound(uint64_t total, uint32_t block_size)
{
    uint64_t r = 0;
    for (const BlockDesc& b : geometry(total, block_size))
        r += rle_capacity(b.len) * 4;  // codes of <= 32 bits
    return r + 64;
}

int bra_gpu_encode_blocks(bra_gpu_ctx_t* c, const uint8_t* d_in, uint64_t total, uint32_t block_size, bra_io_chunk_header_t* d_headers,
                          uint64_t* d_payload_off, uint8_t* d_payload, uint64_t payload_cap, void* stream)
{
    if (!c || !d_in || !total || !block_size || block_size >= (1u << 24) || !d_headers || !d_payload_off || !d_payload)
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t s = cs_;
    g_prof       = c->prof.mask ? &c->prof : nullptr;
    const int rc = encode_impl(c, d_in, geometry(total, block_size), d_headers, d_payload_off, d_payload, payload_cap, s, nullptr);
    g_prof       = nullptr;
    return cs_.finish(rc);
}

int bra_gpu_decode_blocks(bra_gpu_ctx_t* c, const bra_io_chunk_header_t* d_headers, const uint64_t* d_payload_off, const uint8_t* d_payload,
                          uint64_t total, uint32_t block_size, uint8_t* d_out, void* stream)
{
    if (!c || !d_headers || !d_payload_off || !d_payload || !total || !block_size || block_size >= (1u << 24) || !d_out)
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t s = cs_;
    g_prof       = c->prof.mask ? &c->prof : nullptr;
    const int rc = decode_impl(c, d_headers, d_payload_off, d_payload, geometry(total, block_size), d_out, s);
    g_prof       = nullptr;
    return cs_.finish(rc);
}

int bra_gpu_crc32c(bra_gpu_ctx_t* c, const void* d_data, uint64_t len, uint32_t prev, uint32_t* d_crc, void* stream)
{
    if (!c || !d_crc || (len && !d_data))
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t s = cs_;
    if (!crc_stream_device(static_cast<const uint8_t*>(d_data), len, 0, nullptr, prev, d_crc, s))
        return -1;
    return cs_.finish(0);  // NULL stream: complete on return
}

int bra_gpu_chunks_crc32c(bra_gpu_ctx_t* c, const uint8_t* d_data, uint64_t total, uint32_t block_size, const bra_io_chunk_header_t* d_headers,
                          uint32_t prev, uint32_t* d_crc, void* stream)
{
    if (!c || !d_crc || !block_size || (total && (!d_data || !d_headers)))
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t s = cs_;
    if (!crc_stream_device(d_data, total, block_size, reinterpret_cast<const uint8_t*>(d_headers), prev, d_crc, s))
        return -1;
    return cs_.finish(0);
}

uint32_t bra_gpu_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) { return crc32c_combine_host(crc_a, crc_b, len_b); }

uint32_t bra_gpu_entry_crc32c(uint32_t me_crc, uint64_t chunks_size, uint32_t chunks_crc, uint64_t data_size, uint32_t block_size)
{
    const uint64_t num_chunks = block_size ? (data_size + block_size - 1) / block_size : 0;
    const int64_t  tsz        = (int64_t) chunks_size;
    me_crc                    = crc32c_host(&tsz, sizeof tsz, me_crc);
    // bra_crc32c_combine takes a uint32_t length: keep its truncation for parity
    return crc32c_combine_host(me_crc, chunks_crc, (uint32_t) (data_size + num_chunks * sizeof(bra_io_chunk_header_t)));
}

uint64_t bra_gpu_chunks_bound(uint64_t total, uint32_t block_size)
{
    return bra_gpu_payload_bound(total, block_size) + (uint64_t) CHUNK_HDR_DISK * bra_gpu_num_blocks(total, block_size);
}

int bra_gpu_frame_chunks(bra_gpu_ctx_t* c, const bra_io_chunk_header_t* d_headers, const uint64_t* d_payload_off, const uint8_t* d_payload,
                         uint32_t nblocks, uint8_t* d_out, uint64_t out_cap, uint64_t* out_size, void* stream)
{
    if (!c || !d_headers || !d_payload_off || !d_payload || !d_out)
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t s = cs_;
    uint64_t    P = 0;
    if (hipMemcpyAsync(&P, d_payload_off + nblocks, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return -1;
    const uint64_t need = P + (uint64_t) CHUNK_HDR_DISK * nblocks;
    if (out_size)
        *out_size = need;
    if (need > out_cap)
        return -2;
    if (!frame_chunks_device(reinterpret_cast<const uint8_t*>(d_headers), d_payload_off, d_payload, nblocks, d_out, s))
        return -1;
    return cs_.finish(0);
}

int bra_gpu_unframe_chunks(bra_gpu_ctx_t* c, const uint8_t* d_stream, uint64_t stream_size, uint32_t max_chunks, bra_io_chunk_header_t* d_headers,
                           uint64_t* d_payload_off, uint32_t* n_chunks, void* stream)
{
    if (!c || !d_stream || !d_headers || !d_payload_off)
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t s = cs_;
    if (!grow(c->d_word, c->cap_word, 4))
        return -1;
    uint32_t st[2] = {0, 0};
    if (!unframe_chunks_device(d_stream, stream_size, max_chunks, BRA_MAX_CHUNK, reinterpret_cast<uint8_t*>(d_headers), d_payload_off,
                               c->d_word + 1, s) ||
        hipMemcpyAsync(st, c->d_word + 1, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return -1;
    if (n_chunks)
        *n_chunks = st[0];
    if (st[1])
    {
        bra_hip_report(st[1] & 2 ? "chunk header not valid" : "truncated chunk stream (%u records)", st[0]);
        return -1;
    }
    return cs_.finish(0);
}

int bra_gpu_compress_chunks(bra_gpu_ctx_t* c, const uint8_t* d_in, uint64_t data_size, uint32_t block_size, uint8_t* d_out, uint64_t out_cap,
                            uint64_t* out_size, uint32_t* chunks_crc, void* stream)
{
    if (!c || !d_in || !data_size || !block_size || block_size >= (1u << 24) || !d_out)
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t    s  = cs_;
    const auto     hb = geometry(data_size, block_size);
    const uint32_t nb = (uint32_t) hb.size();
    const uint64_t pb = bra_gpu_payload_bound(data_size, block_size);
    if (!grow(c->d_hdr, c->cap_hdr, nb) || !grow(c->d_off, c->cap_off, nb + 1) || !grow(c->d_pay, c->cap_pay, pb) || !grow(c->d_word, c->cap_word, 4))
        return -1;
    g_prof        = c->prof.mask ? &c->prof : nullptr;
    uint64_t P    = 0;
    int      rc   = encode_impl(c, d_in, hb, c->d_hdr, c->d_off, c->d_pay, c->cap_pay, s, &P);
    uint32_t crc  = 0;
    uint64_t need = P + (uint64_t) CHUNK_HDR_DISK * nb;
    if (rc == 0)
    {
        if (out_size)
            *out_size = need;
        if (need > out_cap)
            rc = -2;
    }
    if (rc == 0)
    {
        bool ok;
        {
            BRA_PROF(P_FRAME, s);
            ok = frame_chunks_device(reinterpret_cast<const uint8_t*>(c->d_hdr), c->d_off, c->d_pay, nb, d_out, s);
        }
        if (ok)
        {
            BRA_PROF(P_CRC, s);
            ok = crc_stream_device(d_in, data_size, block_size, reinterpret_cast<const uint8_t*>(c->d_hdr), 0, c->d_word, s);
        }
        if (g_prof)
        {
            prof_bytes(P_FRAME, 2.0 * (double) need);
            prof_bytes(P_CRC, (double) data_size + 268.0 * nb);
        }
        if (!ok || hipMemcpyAsync(&crc, c->d_word, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            rc = -1;
    }
    g_prof = nullptr;
    if (rc != 0)
        return rc;
    if (chunks_crc)
        *chunks_crc = crc;
    return cs_.finish(need < data_size ? 1 : 0);  // 0: not smaller than the input -> STORED (lib_bra_io_file_chunks.c:274-278)
}

static int decompress_chunks_impl(bra_gpu_ctx_t* c, const uint8_t* d_stream, uint64_t stream_size, uint32_t block_size, uint8_t* d_out,
                                  uint64_t out_cap, uint64_t* out_size, uint32_t prev_crc, uint32_t* crc_out, void* stream, bool whole_entry);

int bra_gpu_decompress_chunks(bra_gpu_ctx_t* c, const uint8_t* d_stream, uint64_t stream_size, uint32_t block_size, uint8_t* d_out,
                              uint64_t out_cap, uint64_t* out_size, uint32_t prev_crc, uint32_t* crc_out, void* stream)
{
    return decompress_chunks_impl(c, d_stream, stream_size, block_size, d_out, out_cap, out_size, prev_crc, crc_out, stream, true);
}

// whole_entry: the stream is a whole file entry, so the reference's final safety check applies
// (decoded size must exceed the stream size, lib_bra_io_file_chunks.c:423-427); a front end that
// decodes an entry in several batches checks the total itself.
static int decompress_chunks_impl(bra_gpu_ctx_t* c, const uint8_t* d_stream, uint64_t stream_size, uint32_t block_size, uint8_t* d_out,
                                  uint64_t out_cap, uint64_t* out_size, uint32_t prev_crc, uint32_t* crc_out, void* stream, bool whole_entry)
{
    if (!c || !d_stream || !block_size || block_size >= (1u << 24) || !d_out)
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t    s        = cs_;
    const uint32_t max_recs = (uint32_t) std::min<uint64_t>(stream_size / (CHUNK_HDR_DISK + 1) + 1, 1u << 26);
    if (!grow(c->d_hdr, c->cap_hdr, max_recs) || !grow(c->d_off, c->cap_off, max_recs + 1) || !grow(c->d_word, c->cap_word, 4))
        return -1;
    uint32_t nb = 0;
    if (bra_gpu_unframe_chunks(c, d_stream, stream_size, max_recs, c->d_hdr, c->d_off, &nb, s) != 0)
        return -1;
    if (nb == 0)
    {
        bra_hip_report("corrupted file entry: empty chunk stream");
        return -1;
    }
    std::vector<BlockDesc> caps(nb);
    for (uint32_t b = 0; b < nb; ++b)
        caps[b] = BlockDesc{(uint64_t) b * block_size, block_size, 0};
    uint64_t total = 0;
    std::vector<uint32_t> dsz;
    int      rc    = decode_impl(c, c->d_hdr, c->d_off, d_stream, caps, d_out, s, true, out_cap, &total, &dsz);
    if (out_size)
        *out_size = total;
    if (rc != 0)
        return rc;
    if (whole_entry && total <= stream_size)  // the reference's safety check (:423-427)
    {
        bra_hip_report("corrupted file entry: %llu decoded bytes from %llu", (unsigned long long) total, (unsigned long long) stream_size);
        return -1;
    }
    if (crc_out)
    {
        // The decode loop folds header b then decoded chunk b into me->crc32 (:396-397).  With every
        // chunk but the last at block_size this is one device pass over the packed output; a stream
        // with a short chunk in the middle (accepted like the reference does) is folded chunk by chunk.
        bool regular = true;
        for (uint32_t b = 0; b + 1 < nb; ++b)
            regular = regular && dsz[b] == block_size;
        uint32_t crc = prev_crc;
        if (regular)
        {
            if (!crc_stream_device(d_out, total, block_size, reinterpret_cast<const uint8_t*>(c->d_hdr), prev_crc, c->d_word, s) ||
                hipMemcpyAsync(&crc, c->d_word, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
                return -1;
        }
        else
        {
            uint64_t o = 0;
            for (uint32_t b = 0; b < nb; o += dsz[b], ++b)
                if (!crc_stream_device(d_out + o, dsz[b], dsz[b], reinterpret_cast<const uint8_t*>(c->d_hdr + b), crc, c->d_word, s) ||
                    hipMemcpyAsync(&crc, c->d_word, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
                    return -1;
        }
        *crc_out = crc;
    }
    return cs_.finish(0);
}

// ---- host-buffer forms for the C front end (row f1; frontend/bra_io_file_chunks_gpu.c) ----
// The input is copied into the context's device staging buffer, the device chunk loop runs, and
// the chunk records come back; everything completes before the call returns.
int bra_gpu_compress_chunks_host(bra_gpu_ctx_t* c, const uint8_t* h_in, uint64_t data_size, uint32_t block_size, uint8_t* h_out,
                                 uint64_t out_cap, uint64_t* out_size, uint32_t* chunks_crc)
{
    if (!c || !h_in || !data_size || !block_size || block_size >= (1u << 24) || !h_out)
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    const uint64_t bound = bra_gpu_chunks_bound(data_size, block_size);
    if (!grow(c->d_hin, c->cap_hin, data_size + 16) || !grow(c->d_hout, c->cap_hout, bound + 16) ||
        hipMemcpyAsync(c->d_hin, h_in, data_size, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return -1;
    uint64_t  osz = 0;
    const int rc  = bra_gpu_compress_chunks(c, c->d_hin, data_size, block_size, c->d_hout, c->cap_hout, &osz, chunks_crc, nullptr);
    if (out_size)
        *out_size = osz;
    if (rc < 0)
        return rc;
    if (osz > out_cap)
        return -2;
    if (hipMemcpy(h_out, c->d_hout, osz, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return rc;
}

// ---- pipelined host-buffer chunk compression (row f1 with the copies under the kernels) ----
// Two slots: while slot k's encode runs on the context stream, the next batch's input copy runs on
// copy_in and the previous batch's records come back on copy_out.  The chunk records of a slot are
// framed into the slot's own device buffer, so a later encode never overwrites records not yet
// copied back.  (An optimal prefix code over byte symbols is never longer than the 8-bit code, so a
// block's payload is at most its RLE bytes + 1: the slot buffers use that bound.)
static uint64_t pipe_records_bound(const std::vector<BlockDesc>& hb)
{
    uint64_t r = 64;
    for (const BlockDesc& b : hb)
        r += rle_capacity(b.len) + 16 + CHUNK_HDR_DISK;
    return r;
}

uint64_t bra_gpu_pipe_records_bound(uint64_t total, uint32_t block_size)
{
    return (total && block_size) ? pipe_records_bound(geometry(total, block_size)) : 0;
}

void* bra_gpu_host_alloc(bra_gpu_ctx_t* c, uint64_t bytes)
{
    if (!c || !bytes)
        return nullptr;
    DevGuard dg(c->device);
    void* p = nullptr;
    if (!dg.ok || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess)
    {
        (void) hipGetLastError();
        return nullptr;
    }
    return p;
}

void bra_gpu_host_free(bra_gpu_ctx_t* c, void* p)
{
    if (!c || !p)
        return;
    DevGuard dg(c->device);
    if (c->copy_in)  // a staged input copy may still read the buffer
        (void) hipStreamSynchronize(c->copy_in);
    (void) hipHostFree(p);
}

// The pipeline's streams, pinned mailbox and the slot's events, created on first use.
static bool pipe_init(bra_gpu_ctx_s* c, bra_gpu_ctx_s::PipeSlot& ps)
{
    // The copy streams get the highest priority: HIP maps a process's streams onto a few hardware
    // queues per priority (GPU_MAX_HW_QUEUES), and a kernel queued behind a copy's completion barrier
    // on a shared queue waits for that copy -- a normal-priority copy stream sharing a queue with the
    // encode stream made batch k's kernels wait for batch k + 1's input (scripts/micro/ev_wait.py).
    int least = 0, greatest = 0;
    if (!c->copy_in && (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
                        hipStreamCreateWithPriority(&c->copy_in, hipStreamNonBlocking, greatest) != hipSuccess ||
                        hipStreamCreateWithPriority(&c->copy_out, hipStreamNonBlocking, greatest) != hipSuccess))
        return false;
    if (!c->h_pipe_mail && hipHostMalloc(&c->h_pipe_mail, 4 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess)
    {
        c->h_pipe_mail = nullptr;
        return false;
    }
    return (ps.ev_in || hipEventCreateWithFlags(&ps.ev_in, hipEventDisableTiming) == hipSuccess) &&
           (ps.ev_done || hipEventCreateWithFlags(&ps.ev_done, hipEventDisableTiming) == hipSuccess);
}

// The slot's input copy on the copy stream, after the device has finished the slot's previous batch
// (its BWT and CRC read d_in; ev_done is recorded after both).  The buffer only grows while the slot
// holds no batch.
static bool pipe_copy_in(bra_gpu_ctx_s* c, bra_gpu_ctx_s::PipeSlot& ps, const uint8_t* h_in, uint64_t data_size)
{
    if (data_size + 16 > ps.cap_in && (ps.state != 0 || !grow(ps.d_in, ps.cap_in, data_size + 16)))
        return false;
    return hipStreamWaitEvent(c->copy_in, ps.ev_done, 0) == hipSuccess &&
           hipMemcpyAsync(ps.d_in, h_in, data_size, hipMemcpyHostToDevice, c->copy_in) == hipSuccess &&
           hipEventRecord(ps.ev_in, c->copy_in) == hipSuccess;
}

int bra_gpu_compress_chunks_stage(bra_gpu_ctx_t* c, int slot, const uint8_t* h_in, uint64_t data_size)
{
    if (!c || slot < 0 || slot > 1 || !h_in || !data_size)
        return -1;
    auto& ps = c->pipe[slot];
    if (ps.staged)
        return -1;  // submit the staged batch first
    DevGuard dg(c->device);
    if (!dg.ok || !pipe_init(c, ps) || !pipe_copy_in(c, ps, h_in, data_size))
        return -1;
    ps.staged  = true;
    ps.st_ptr  = h_in;
    ps.st_size = data_size;
    return 0;
}

int bra_gpu_compress_chunks_submit(bra_gpu_ctx_t* c, int slot, const uint8_t* h_in, uint64_t data_size, uint32_t block_size)
{
    if (!c || slot < 0 || slot > 1 || !h_in || !data_size || !block_size || block_size >= (1u << 24))
        return -1;
    auto& ps = c->pipe[slot];
    if (ps.state != 0)
        return -1;  // collect the slot first
    if (ps.staged && (ps.st_ptr != h_in || ps.st_size != data_size))
        return -1;  // not the batch staged for this slot
    DevGuard dg(c->device);
    if (!dg.ok || !pipe_init(c, ps))
        return -1;
    const bool     staged = ps.staged;
    ps.staged             = false;
    const auto     hb     = geometry(data_size, block_size);
    const uint32_t nb     = (uint32_t) hb.size();
    const uint64_t rb     = pipe_records_bound(hb);
    hipStream_t    s      = c->stream;
    if (!grow(ps.d_out, ps.cap_out, rb + 16) || !grow(c->d_hdr, c->cap_hdr, nb) || !grow(c->d_off, c->cap_off, nb + 1) ||
        !grow(c->d_pay, c->cap_pay, rb) || !grow(c->d_word, c->cap_word, 4))
        return -1;
    if ((!staged && !pipe_copy_in(c, ps, h_in, data_size)) || hipStreamWaitEvent(s, ps.ev_in, 0) != hipSuccess ||
        (c->caller_pending && hipStreamWaitEvent(s, c->caller_ev, 0) != hipSuccess))
        return -1;
    g_prof = c->prof.mask ? &c->prof : nullptr;
    int rc = encode_impl(c, ps.d_in, hb, c->d_hdr, c->d_off, c->d_pay, c->cap_pay, s, nullptr);
    g_prof = nullptr;
    uint64_t* mail = c->h_pipe_mail + 2 * slot;
    if (rc == 0 &&
        (!frame_chunks_device(reinterpret_cast<const uint8_t*>(c->d_hdr), c->d_off, c->d_pay, nb, ps.d_out, s) ||
         !crc_stream_device(ps.d_in, data_size, block_size, reinterpret_cast<const uint8_t*>(c->d_hdr), 0, c->d_word, s) ||
         hipMemcpyAsync(mail, c->d_off + nb, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
         hipMemcpyAsync(mail + 1, c->d_word, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipEventRecord(ps.ev_done, s) != hipSuccess))
        rc = -1;
    // the caller may refill h_in once this returns (the encode's host waits came after the copy;
    // this wait is for the error paths and says so explicitly)
    if (hipEventSynchronize(ps.ev_in) != hipSuccess)
        rc = -1;
    if (rc != 0)
    {
        (void) hipStreamSynchronize(s);
        return -1;
    }
    ps.data_size = data_size;
    ps.nb        = nb;
    ps.state     = 1;
    return 0;
}

int bra_gpu_compress_chunks_collect(bra_gpu_ctx_t* c, int slot, uint8_t* h_out, uint64_t out_cap, uint64_t* out_size, uint32_t* chunks_crc)
{
    if (!c || slot < 0 || slot > 1)
        return -1;
    auto&    ps = c->pipe[slot];
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    if (!h_out && ps.staged)
    {
        // a drain (no output buffer) also drops the slot's staged input copy
        (void) hipStreamSynchronize(c->copy_in);
        ps.staged = false;
    }
    if (ps.state != 1)
        return -1;
    if (hipEventSynchronize(ps.ev_done) != hipSuccess)
    {
        ps.state = 0;
        return -1;
    }
    const uint64_t* mail = c->h_pipe_mail + 2 * slot;
    const uint64_t  need = mail[0] + (uint64_t) CHUNK_HDR_DISK * ps.nb;
    if (out_size)
        *out_size = need;
    if (chunks_crc)
        *chunks_crc = (uint32_t) mail[1];
    if (h_out && need > out_cap)
        return -2;  // the batch stays in the slot: collect again with a larger buffer (or drain it)
    ps.state = 0;
    if (!h_out)
        return -1;
    if (hipMemcpyAsync(h_out, ps.d_out, need, hipMemcpyDeviceToHost, c->copy_out) != hipSuccess || hipStreamSynchronize(c->copy_out) != hipSuccess)
        return -1;
    return need < ps.data_size ? 1 : 0;  // 0: not smaller than the input -> STORED (lib_bra_io_file_chunks.c:274-278)
}

int bra_gpu_decompress_chunks_host(bra_gpu_ctx_t* c, const uint8_t* h_stream, uint64_t stream_size, uint32_t block_size, uint8_t* h_out,
                                   uint64_t out_cap, uint64_t* out_size, uint32_t prev_crc, uint32_t* crc_out, int whole_entry)
{
    if (!c || !h_stream || !stream_size || !block_size || block_size >= (1u << 24) || !h_out)
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    if (!grow(c->d_hin, c->cap_hin, stream_size + 16) || !grow(c->d_hout, c->cap_hout, out_cap + 16) ||
        hipMemcpyAsync(c->d_hin, h_stream, stream_size, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return -1;
    uint64_t  osz = 0;
    const int rc  = decompress_chunks_impl(c, c->d_hin, stream_size, block_size, c->d_hout, out_cap, &osz, prev_crc, crc_out, nullptr,
                                           whole_entry != 0);
    if (out_size)
        *out_size = osz;
    if (rc != 0)
        return rc;
    if (hipMemcpy(h_out, c->d_hout, osz, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return 0;
}

int bra_gpu_chunks_crc32c_shard(bra_gpu_ctx_t* c, const uint8_t* d_data, uint64_t total, uint32_t block_size, const bra_io_chunk_header_t* d_headers,
                                uint64_t first_chunk, uint64_t chunk_stride, uint64_t global_total, uint32_t prev, int with_init, uint32_t* d_crc,
                                void* stream)
{
    if (!c || !d_crc || !block_size || !chunk_stride || (total && (!d_data || !d_headers)))
        return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t s = cs_;
    if (!crc_stream_shard_device(d_data, total, block_size, reinterpret_cast<const uint8_t*>(d_headers), first_chunk, chunk_stride, global_total,
                                 prev, with_init != 0, d_crc, s))
        return -1;
    return cs_.finish(0);
}

int bra_gpu_assemble_shards(bra_gpu_ctx_t* c, uint32_t nparts, const bra_io_chunk_header_t* const* d_headers, const uint64_t* const* d_payload_off,
                            const uint8_t* const* d_payload, const uint32_t* nblocks, int round_robin, bra_io_chunk_header_t* d_headers_out,
                            uint64_t* d_payload_off_out, uint8_t* d_payload_out, uint64_t payload_cap, void* stream)
{
    if (!c || nparts == 0 || nparts > MAX_SHARDS || !d_headers || !d_payload_off || !d_payload || !nblocks || !d_headers_out ||
        !d_payload_off_out || !d_payload_out)
        return -1;
    ShardParts P{};
    P.n           = nparts;
    P.round_robin = round_robin ? 1u : 0u;
    uint64_t nb   = 0;
    for (uint32_t p = 0; p < nparts; ++p)
    {
        if (!d_headers[p] || !d_payload_off[p] || (!d_payload[p] && nblocks[p]))
            return -1;
        P.hdr[p]   = reinterpret_cast<const uint8_t*>(d_headers[p]);
        P.off[p]   = d_payload_off[p];
        P.pay[p]   = d_payload[p];
        P.first[p] = (uint32_t) nb;
        nb += nblocks[p];
    }
    P.first[nparts] = (uint32_t) nb;
    if (nb == 0 || nb >= (1ull << 31))
        return -1;
    if (round_robin)
        for (uint32_t p = 0; p < nparts; ++p)  // part p must hold exactly the blocks g = p (mod nparts)
            if ((uint64_t) nblocks[p] != (nb > p ? (nb - p + nparts - 1) / nparts : 0))
                return -1;
    DevGuard dg(c->device);
    if (!dg.ok)
        return -1;
    CallStream cs_(c, stream);
    hipStream_t s = cs_;
    // d_word: [3] overflow flag, [4..5] the payload size needed (u64)
    if (!grow(c->d_word, c->cap_word, 8) ||
        !assemble_shards_device(P, (uint32_t) nb, reinterpret_cast<uint8_t*>(d_headers_out), d_payload_off_out, d_payload_out, payload_cap,
                                c->d_word + 3, reinterpret_cast<uint64_t*>(c->d_word + 4), s))
        return -1;
    if (stream)
        return 0;  // asynchronous: an overflow shows as d_payload_off_out[nb] == UINT64_MAX
    uint32_t err = 1;
    if (hipMemcpyAsync(&err, c->d_word + 3, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return -1;
    // on overflow, leave the size needed where the caller reads the payload size (offsets[N])
    if (err && hipMemcpyAsync(d_payload_off_out + nb, c->d_word + 4, 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
        return -1;
    return cs_.finish(err ? -2 : 0);
}

const void* bra_gpu_stage_ptr(bra_gpu_ctx_t* c, int stage)
{
    if (!c)
        return nullptr;
    switch (stage)
    {
    case 0: return c->d_L;
    case 1: return c->d_mtf;
    case 2: return c->d_rle;
    case 3: return c->d_enc_rle_base;  // RLE output bases of the last batch encode
    case 4: return c->d_rle_size;
    case 5: return bwt_sa(c->bwt);  // BWT suffix-array slots of the last batch encode (diagnostics)
    default: return nullptr;
    }
}

// Diagnostics: re-run the job phase of the last batch encode `reps` times (each time with the jobs'
// inputs in another order when shuffle_seed != 0) and audit it.  Returns the failing jobs summed
// over the runs, -1 on an error.
int bra_gpu_debug_rerun_jobs(bra_gpu_ctx_t* c, int reps, unsigned shuffle_seed)
{
    if (!c)
        return -1;
    DevGuard dg(c->device);
    return bwt_debug_rerun_jobs(c->bwt, reps, c->stream, shuffle_seed);
}

const char* bra_gpu_version(void) { return "bra_hip 0.1.0 (gfx950)"; }

void bra_gpu_prof_enable(bra_gpu_ctx_t* c, uint64_t mask)
{
    if (c)
        c->prof.mask = mask;
}

void bra_gpu_prof_reset(bra_gpu_ctx_t* c)
{
    if (c)
        c->prof.reset();
}

int bra_gpu_prof_read(bra_gpu_ctx_t* c, int slot, const char** name, double* total_ms, uint32_t* launches, double* bytes)
{
    if (!c)
        return 0;
    c->prof.collect();
    if (slot >= 0 && slot < P_NSLOT)
    {
        if (name)
            *name = prof_name(slot);
        if (total_ms)
            *total_ms = c->prof.ms[slot];
        if (launches)
            *launches = c->prof.launches[slot];
        if (bytes)
            *bytes = c->prof.bytes[slot];
    }
    return P_NSLOT;
}

}  // extern "C"

// =================================================================================================
// Part 1: the reference encoder ABI on lazily created contexts of the caller's current device
// =================================================================================================
namespace {

// The reference encoders are reentrant (no globals), so calls from several host threads must not
// queue behind one another: each call leases a context of the calling thread's current HIP device
// from that device's pool (creating one when all are busy) and returns it afterwards.  Contexts live
// until process exit; a pool grows to the number of threads that ever called concurrently.
constexpr int MAX_DEVICES = 64;

struct CtxPool
{
    std::mutex                  mu;
    std::vector<bra_gpu_ctx_s*> idle;
};
CtxPool g_pools[MAX_DEVICES];

struct CtxLease
{
    bra_gpu_ctx_s* ctx = nullptr;
    int            dev = -1;
    CtxLease()
    {
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEVICES)
        {
            (void) hipGetLastError();
            bra_hip_report("no usable HIP device for the block codec");
            dev = -1;
            return;
        }
        {
            std::lock_guard<std::mutex> lk(g_pools[dev].mu);
            if (!g_pools[dev].idle.empty())
            {
                ctx = g_pools[dev].idle.back();
                g_pools[dev].idle.pop_back();
                return;
            }
        }
        auto* c = new bra_gpu_ctx_s();
        if (!ctx_init(c, dev))
        {
            bra_hip_report("unable to create a block-codec context on HIP device %d", dev);
            ctx_free(c);
            delete c;
            return;
        }
        ctx = c;
    }
    ~CtxLease()
    {
        if (!ctx)
            return;
        std::lock_guard<std::mutex> lk(g_pools[dev].mu);
        g_pools[dev].idle.push_back(ctx);
    }
    CtxLease(const CtxLease&)            = delete;
    CtxLease& operator=(const CtxLease&) = delete;
};

bool upload(bra_gpu_ctx_s* c, const uint8_t* buf, uint64_t n)
{
    if (!grow(c->d_io, c->cap_io, n + 64))
        return false;
    BRA_HIP_CHECK(hipMemcpyAsync(c->d_io, buf, n, hipMemcpyHostToDevice, c->stream));
    return true;
}

bool download(bra_gpu_ctx_s* c, void* dst, const void* src, uint64_t n)
{
    if (n)
        BRA_HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream));
    BRA_HIP_CHECK(hipStreamSynchronize(c->stream));
    return true;
}

std::vector<BlockDesc> one_block(uint64_t n) { return {BlockDesc{0, (uint32_t) n, 0}}; }

}  // namespace

extern "C" {

bool bra_bwt_encode2(const uint8_t* buf, const bra_bwt_index_t buf_size, bra_bwt_index_t* primary_index, uint8_t* out_buf)
{
    if (!buf || !buf_size || !primary_index || !out_buf)
        return false;
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    if (!c || !upload(c, buf, buf_size))
        return false;
    auto hb = one_block(buf_size);
    if (!ensure_block_arrays(c, 1) || !grow(c->d_L, c->cap_L, (uint64_t) buf_size + 16))
        return false;
    if (buf_size >= (1u << 24))  // past the batched path's 24-bit rotation indices
        return bwt_encode_large(c->d_io, buf_size, c->d_L, c->d_pi, c->stream) && download(c, primary_index, c->d_pi, 4) &&
               download(c, out_buf, c->d_L, buf_size);
    if (hipMemcpyAsync(c->d_blocks, hb.data(), sizeof(BlockDesc), hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return false;
    if (!bwt_encode_device(c->bwt, c->d_io, c->d_blocks, hb.data(), 1, c->d_L, c->d_pi, c->stream))
        return false;
    return download(c, primary_index, c->d_pi, 4) && download(c, out_buf, c->d_L, buf_size);
}

uint8_t* bra_bwt_encode(const uint8_t* buf, const bra_bwt_index_t buf_size, bra_bwt_index_t* primary_index)
{
    uint8_t* out = (uint8_t*) malloc(buf_size);
    if (!out)
        return nullptr;
    if (!bra_bwt_encode2(buf, buf_size, primary_index, out))
    {
        free(out);
        return nullptr;
    }
    return out;
}

void bra_bwt_decode2(const uint8_t* buf, const bra_bwt_index_t buf_size, const bra_bwt_index_t primary_index, bra_bwt_index_t* transform,
                     uint8_t* out_buf)
{
    if (!buf || !buf_size || !out_buf || primary_index >= buf_size)
        return;
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    if (!c || !upload(c, buf, buf_size))
        return;
    auto hb = one_block(buf_size);
    if (!ensure_block_arrays(c, 1) || !grow(c->d_L, c->cap_L, (uint64_t) buf_size + 16))
        return;
    if (hipMemcpyAsync(c->d_blocks, hb.data(), sizeof(BlockDesc), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(c->d_pi, &primary_index, 4, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return;
    if (!ibwt_device(c->ib, c->d_io, c->d_pi, c->d_blocks, hb.data(), 1, c->d_L, c->stream, transform != nullptr))
        return;
    if (transform)
        (void) download(c, transform, c->ib.T, (uint64_t) buf_size * 4);  // the LF transform, as the reference leaves it
    (void) download(c, out_buf, c->d_L, buf_size);
}

uint8_t* bra_bwt_decode(const uint8_t* buf, const bra_bwt_index_t buf_size, const bra_bwt_index_t primary_index)
{
    if (!buf || !buf_size || primary_index >= buf_size)
        return nullptr;
    uint8_t* out = (uint8_t*) malloc(buf_size);
    if (!out)
        return nullptr;
    bra_bwt_decode2(buf, buf_size, primary_index, nullptr, out);
    return out;
}

bool bra_mtf_encode2(const uint8_t* buf, const size_t buf_size, uint8_t* out_buf)
{
    if (!buf || !buf_size || !out_buf || buf_size >= (1ull << 31))
        return false;
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    if (!c || !upload(c, buf, buf_size) || !grow(c->d_mtf, c->cap_mtf, (uint64_t) buf_size + 16))
        return false;
    // blocks of 2^24 bytes or more: the segment scan is exact at any length; start tables whose
    // last occurrences pass 24 bits take the two-pass sort (mtf.hip start_table_dword)
    std::vector<BlockDesc> hb{BlockDesc{0, (uint32_t) buf_size, 0}};
    if (!mtf_encode_device(c->mtf, c->d_io, c->d_mtf, hb.data(), 1, c->stream))
        return false;
    return download(c, out_buf, c->d_mtf, buf_size);
}

uint8_t* bra_mtf_encode(const uint8_t* buf, const size_t buf_size)
{
    uint8_t* out = (uint8_t*) malloc(buf_size ? buf_size : 1);
    if (!out)
        return nullptr;
    if (!bra_mtf_encode2(buf, buf_size, out))
    {
        free(out);
        return nullptr;
    }
    return out;
}

void bra_mtf_decode2(const uint8_t* buf, const size_t buf_size, uint8_t* out_buf)
{
    if (!buf || !buf_size || !out_buf || buf_size >= (1ull << 31))
        return;
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    if (!c || !upload(c, buf, buf_size) || !grow(c->d_mtf, c->cap_mtf, (uint64_t) buf_size + 16) ||
        !grow(c->d_tmp, c->cap_tmp, (uint64_t) buf_size + 16))
        return;
    std::vector<BlockDesc> hb{BlockDesc{0, (uint32_t) buf_size, 0}};
    if (!mtf_decode_device(c->mtf, c->d_io, c->d_mtf, c->d_tmp, hb.data(), 1, c->stream))
        return;
    (void) download(c, out_buf, c->d_mtf, buf_size);
}

uint8_t* bra_mtf_decode(const uint8_t* buf, const size_t buf_size)
{
    if (!buf || !buf_size)
        return nullptr;
    uint8_t* out = (uint8_t*) malloc(buf_size);
    if (!out)
        return nullptr;
    bra_mtf_decode2(buf, buf_size, out);
    return out;
}

bool bra_rle_encode(const uint8_t* buf, const size_t buf_size, uint8_t** out_buf, size_t* out_buf_size)
{
    if (out_buf)
        *out_buf = nullptr;
    if (out_buf_size)
        *out_buf_size = 0;
    if (!buf || !out_buf || !out_buf_size || buf_size == 0 || buf_size >= (1ull << 31))
        return false;
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    if (!c || !upload(c, buf, buf_size) || !ensure_block_arrays(c, 1))
        return false;
    const uint64_t cap = rle_capacity((uint32_t) buf_size);
    if (!grow(c->d_rle, c->cap_rle, cap + 16))
        return false;
    const uint64_t zero = 0;
    if (hipMemcpyAsync(c->d_rle_base, &zero, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return false;
    std::vector<BlockDesc> hb{BlockDesc{0, (uint32_t) buf_size, 0}};
    if (!rle_encode_device(c->rle, c->d_io, hb.data(), 1, c->d_rle_base, c->d_rle, c->d_rle_size, c->d_hist, c->stream))
        return false;
    uint32_t rs = 0;
    if (!download(c, &rs, c->d_rle_size, 4) || rs == 0)
        return false;
    uint8_t* b = (uint8_t*) malloc(rs);
    if (!b)
        return false;
    if (!download(c, b, c->d_rle, rs))
    {
        free(b);
        return false;
    }
    *out_buf      = b;
    *out_buf_size = rs;
    return true;
}

static bool rle_decode_one(bra_gpu_ctx_s* c, const uint8_t* buf, size_t buf_size, uint32_t* dec_size, bool expand)
{
    if (!upload(c, buf, buf_size) || !ensure_block_arrays(c, 1))
        return false;
    const uint64_t out_cap = expand ? (uint64_t) buf_size * 64 + 64 : 0;  // a 2-byte run block expands to <= 128 bytes
    if (!grow(c->d_tmp, c->cap_tmp, std::max<uint64_t>(out_cap, 16)))
        return false;
    const uint64_t zero = 0, cap = out_cap;
    const uint32_t sz   = (uint32_t) buf_size;
    if (hipMemcpyAsync(c->d_rle_base, &zero, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(c->d_rle_cap, &cap, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(c->d_aux, &zero, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(c->d_rle_size, &sz, 4, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return false;
    if (!rle_decode_device(c->rle, &sz, c->d_io, c->d_rle_base, c->d_rle_size, 1, c->d_tmp, c->d_aux, c->d_rle_cap, c->d_status, c->stream))
        return false;
    return download(c, dec_size, c->d_status, 4);
}

size_t bra_rle_decode_compute_size(const uint8_t* buf, const size_t buf_size)
{
    if (!buf || buf_size == 0 || buf_size >= (1ull << 31))
        return 0;
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    uint32_t                    s = 0;
    if (!c || !rle_decode_one(c, buf, buf_size, &s, false))
        return 0;
    return s;
}

bool bra_rle_decode(const uint8_t* buf, const size_t buf_size, uint8_t** out_buf, size_t* out_buf_size)
{
    if (out_buf)
        *out_buf = nullptr;
    if (out_buf_size)
        *out_buf_size = 0;
    if (!buf || !out_buf || !out_buf_size || buf_size == 0 || buf_size >= (1ull << 31))
        return false;
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    uint32_t                    s = 0;
    if (!c || !rle_decode_one(c, buf, buf_size, &s, true) || s == 0)
        return false;
    uint8_t* b = (uint8_t*) malloc(s);
    if (!b)
        return false;
    if (!download(c, b, c->d_tmp, s))
    {
        free(b);
        return false;
    }
    *out_buf      = b;
    *out_buf_size = s;
    return true;
}

bra_huffman_chunk_t* bra_huffman_encode(const uint8_t* buf, const uint32_t buf_size)
{
    if (!buf || buf_size == 0)
    {
        bra_hip_report("unable to huffman encode");
        return nullptr;
    }
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    if (!c || !upload(c, buf, buf_size) || !ensure_block_arrays(c, 1) || !grow(c->d_off, c->cap_off, 4))
        return nullptr;
    std::vector<BlockDesc> hb{BlockDesc{0, buf_size, 0}};
    if (!histogram_device(c->hist_tiling, c->d_io, hb.data(), 1, c->d_hist, c->stream))
        return nullptr;
    if (hipMemcpyAsync(c->d_rle_size, &buf_size, 4, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return nullptr;
    uint64_t cap = (uint64_t) buf_size * 4 + 64, total = 0;
    for (int attempt = 0; attempt < 2; ++attempt)
    {
        if (!grow(c->d_pay, c->cap_pay, cap))
            return nullptr;
        if (huff_encode_device(c->huf, c->d_io, hb.data(), 1, c->d_hist, c->d_rle_size, c->d_meta, c->d_off, c->d_pay, c->cap_pay, &total,
                               c->stream))
            break;
        if (total + 8 <= c->cap_pay || attempt == 1)
            return nullptr;
        cap = total + 64;
    }
    auto* out = (bra_huffman_chunk_t*) malloc(sizeof(bra_huffman_chunk_t));
    if (!out)
        return nullptr;
    out->data = nullptr;
    if (!download(c, &out->meta, c->d_meta, sizeof(bra_huffman_t)))
    {
        free(out);
        return nullptr;
    }
    out->data = (uint8_t*) malloc(out->meta.encoded_size ? out->meta.encoded_size : 1);
    if (!out->data || !download(c, out->data, c->d_pay, out->meta.encoded_size))
    {
        free(out->data);
        free(out);
        return nullptr;
    }
    return out;
}

uint8_t* bra_huffman_decode(const bra_huffman_t* meta, const uint8_t* data, uint32_t* out_size)
{
    if (out_size)
        *out_size = 0;
    if (!meta || !data || !out_size)
        return nullptr;
    CtxLease       lease;
    bra_gpu_ctx_s* c = lease.ctx;
    if (!c || !ensure_block_arrays(c, 1) || !grow(c->d_off, c->cap_off, 4))
        return nullptr;
    if (!upload(c, data, meta->encoded_size) || !grow(c->d_tmp, c->cap_tmp, (uint64_t) meta->orig_size + 16))
        return nullptr;
    const uint64_t zero = 0;
    if (hipMemcpyAsync(c->d_meta, meta, sizeof(bra_huffman_t), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(c->d_off, &zero, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(c->d_rle_base, &zero, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return nullptr;
    const uint32_t esz = meta->encoded_size;
    if (!huff_decode_device(c->huf, c->d_meta, &esz, 1, c->d_io, c->d_off, c->d_tmp, c->d_rle_base, c->d_status, c->stream))
        return nullptr;
    uint32_t st = 1;
    if (!download(c, &st, c->d_status, 4) || st)
    {
        bra_hip_report("huffman decode error: invalid code sequence");
        return nullptr;
    }
    uint8_t* out = (uint8_t*) malloc(meta->orig_size ? meta->orig_size : 1);
    if (!out || !download(c, out, c->d_tmp, meta->orig_size))
    {
        free(out);
        return nullptr;
    }
    *out_size = meta->orig_size;
    return out;
}

void bra_huffman_chunk_free(bra_huffman_chunk_t* chunk)
{
    if (!chunk)
        return;
    free(chunk->data);
    free(chunk);
}

}  // extern "C"
