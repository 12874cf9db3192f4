"""br-archive_amd -- host-side mirror of br-archive's encoder interface on the MI355X block codec.

The product is ``libbra_hip.so`` (C-ABI in ``include/bra_hip.h``; HIP kernels for gfx950 under
``csrc/``).  This module only binds it:

* the reference's encoder functions (``src/encoders/bra_{bwt,mtf,rle,huffman}.h``) with the same
  names, argument meaning and failure behaviour (``None``/``False`` where the C function returns
  ``NULL``/``false``), one block per call on host buffers;
* :class:`BlockCodec`, the batched device-resident API (``bra_gpu_encode_blocks`` /
  ``bra_gpu_decode_blocks``) on torch tensors that already live in HBM.

There is no CPU implementation here: importing raises if the HIP library is missing or was not
built, and every call runs on the GPU.  (The CPU restatement used to check results lives in the
top-level ``oracle/`` package, which this package never imports.)

Import with ``importlib.import_module("br-archive_amd")`` (the directory name carries a hyphen).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

HERE = os.path.dirname(os.path.abspath(__file__))
# BRA_HIP_LIB: an alternative build of the same library (measurement variants built by
# scripts/build_variants.sh); the default is the in-tree product library.
LIB_PATH = os.environ.get("BRA_HIP_LIB") or os.path.join(HERE, "libbra_hip.so")
SYNTH_PATH = os.path.join(HERE, "libbra_synth.so")

# Exported symbols of include/bra_hip.h (checked by tests/test_abi.py against the header).
ABI_SYMBOLS = (
    "bra_bwt_encode", "bra_bwt_encode2", "bra_bwt_decode", "bra_bwt_decode2",
    "bra_mtf_encode", "bra_mtf_encode2", "bra_mtf_decode", "bra_mtf_decode2",
    "bra_rle_encode", "bra_rle_decode_compute_size", "bra_rle_decode",
    "bra_huffman_encode", "bra_huffman_decode", "bra_huffman_chunk_free",
    "bra_gpu_ctx_create", "bra_gpu_ctx_destroy", "bra_gpu_num_blocks", "bra_gpu_payload_bound",
    "bra_gpu_encode_blocks", "bra_gpu_decode_blocks", "bra_gpu_stage_ptr", "bra_gpu_version", "bra_gpu_selftest",
    "bra_gpu_prof_enable", "bra_gpu_prof_reset", "bra_gpu_prof_read",
    "bra_gpu_crc32c", "bra_gpu_chunks_crc32c", "bra_gpu_crc32c_combine", "bra_gpu_entry_crc32c", "bra_gpu_chunks_bound",
    "bra_gpu_pipe_records_bound",
    "bra_gpu_frame_chunks", "bra_gpu_unframe_chunks", "bra_gpu_compress_chunks", "bra_gpu_decompress_chunks",
    "bra_gpu_compress_chunks_host", "bra_gpu_decompress_chunks_host",
    "bra_gpu_chunks_crc32c_shard", "bra_gpu_assemble_shards",
    "bra_gpu_debug_rerun_jobs", "bra_gpu_sortnet_selftest",
    "bra_gpu_host_alloc", "bra_gpu_host_free", "bra_gpu_compress_chunks_stage", "bra_gpu_compress_chunks_submit", "bra_gpu_compress_chunks_collect",
)
MAX_CHUNK_SIZE = 256 * 1024  # BRA_MAX_CHUNK_SIZE (src/lib_bra_defs.h:93): the .BRa chunk size

SYNTH_TEXT, SYNTH_RANDOM, SYNTH_SYM16, SYNTH_TILED = 0, 1, 2, 3
HEADER_BYTES = 268  # in-memory bra_io_chunk_header_t (pi u32 + packed bra_huffman_t)


class HuffmanMeta(C.Structure):
    """bra_huffman_t (src/lib_bra_types.h:51-56), packed."""

    _pack_ = 1
    _fields_ = [("lengths", C.c_uint8 * 256), ("orig_size", C.c_uint32), ("encoded_size", C.c_uint32)]


class _HuffmanChunk(C.Structure):
    """bra_huffman_chunk_t (src/encoders/bra_huffman.h:13-17)."""

    _fields_ = [("meta", HuffmanMeta), ("data", C.c_void_p)]


assert C.sizeof(HuffmanMeta) == 264 and _HuffmanChunk.data.offset == 264


@dataclass
class HuffmanChunk:
    lengths: bytes
    orig_size: int
    encoded_size: int
    data: bytes


def _load() -> C.CDLL:
    # One HIP runtime per process: torch ships its own libamdhip64 (same SONAME).  Loading torch
    # first makes libbra_hip.so bind to that copy instead of opening a second runtime that could
    # no longer see the GPUs.  Without torch the library uses /opt/rocm's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make -C br-archive_amd` (or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    u8p, u32p, vp = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.c_void_p
    lib.bra_bwt_encode2.argtypes = [u8p, C.c_uint32, u32p, u8p]
    lib.bra_bwt_encode2.restype = C.c_bool
    lib.bra_bwt_decode2.argtypes = [u8p, C.c_uint32, C.c_uint32, u32p, u8p]
    lib.bra_bwt_decode2.restype = None
    lib.bra_mtf_encode2.argtypes = [u8p, C.c_size_t, u8p]
    lib.bra_mtf_encode2.restype = C.c_bool
    lib.bra_mtf_decode2.argtypes = [u8p, C.c_size_t, u8p]
    lib.bra_mtf_decode2.restype = None
    lib.bra_rle_encode.argtypes = [u8p, C.c_size_t, C.POINTER(vp), C.POINTER(C.c_size_t)]
    lib.bra_rle_encode.restype = C.c_bool
    lib.bra_rle_decode.argtypes = [u8p, C.c_size_t, C.POINTER(vp), C.POINTER(C.c_size_t)]
    lib.bra_rle_decode.restype = C.c_bool
    lib.bra_rle_decode_compute_size.argtypes = [u8p, C.c_size_t]
    lib.bra_rle_decode_compute_size.restype = C.c_size_t
    lib.bra_huffman_encode.argtypes = [u8p, C.c_uint32]
    lib.bra_huffman_encode.restype = C.POINTER(_HuffmanChunk)
    lib.bra_huffman_decode.argtypes = [C.POINTER(HuffmanMeta), u8p, u32p]
    lib.bra_huffman_decode.restype = vp
    lib.bra_huffman_chunk_free.argtypes = [C.POINTER(_HuffmanChunk)]
    lib.bra_huffman_chunk_free.restype = None
    lib.bra_gpu_ctx_create.argtypes = [C.c_int]
    lib.bra_gpu_ctx_create.restype = vp
    lib.bra_gpu_ctx_destroy.argtypes = [vp]
    lib.bra_gpu_ctx_destroy.restype = None
    lib.bra_gpu_num_blocks.argtypes = [C.c_uint64, C.c_uint32]
    lib.bra_gpu_num_blocks.restype = C.c_uint32
    lib.bra_gpu_payload_bound.argtypes = [C.c_uint64, C.c_uint32]
    lib.bra_gpu_payload_bound.restype = C.c_uint64
    lib.bra_gpu_encode_blocks.argtypes = [vp, vp, C.c_uint64, C.c_uint32, vp, vp, vp, C.c_uint64, vp]
    lib.bra_gpu_encode_blocks.restype = C.c_int
    lib.bra_gpu_decode_blocks.argtypes = [vp, vp, vp, vp, C.c_uint64, C.c_uint32, vp, vp]
    lib.bra_gpu_decode_blocks.restype = C.c_int
    lib.bra_gpu_stage_ptr.argtypes = [vp, C.c_int]
    lib.bra_gpu_stage_ptr.restype = vp
    lib.bra_gpu_prof_enable.argtypes = [vp, C.c_uint64]
    lib.bra_gpu_prof_enable.restype = None
    lib.bra_gpu_prof_reset.argtypes = [vp]
    lib.bra_gpu_prof_reset.restype = None
    lib.bra_gpu_prof_read.argtypes = [vp, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(C.c_uint32),
                                      C.POINTER(C.c_double)]
    lib.bra_gpu_prof_read.restype = C.c_int
    lib.bra_gpu_version.argtypes = []
    lib.bra_gpu_version.restype = C.c_char_p
    lib.bra_gpu_selftest.argtypes = []
    lib.bra_gpu_selftest.restype = C.c_int
    u64p = C.POINTER(C.c_uint64)
    lib.bra_gpu_crc32c.argtypes = [vp, vp, C.c_uint64, C.c_uint32, vp, vp]
    lib.bra_gpu_crc32c.restype = C.c_int
    lib.bra_gpu_chunks_crc32c.argtypes = [vp, vp, C.c_uint64, C.c_uint32, vp, C.c_uint32, vp, vp]
    lib.bra_gpu_chunks_crc32c.restype = C.c_int
    lib.bra_gpu_crc32c_combine.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
    lib.bra_gpu_crc32c_combine.restype = C.c_uint32
    lib.bra_gpu_entry_crc32c.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32]
    lib.bra_gpu_entry_crc32c.restype = C.c_uint32
    lib.bra_gpu_chunks_bound.argtypes = [C.c_uint64, C.c_uint32]
    lib.bra_gpu_chunks_bound.restype = C.c_uint64
    lib.bra_gpu_pipe_records_bound.argtypes = [C.c_uint64, C.c_uint32]
    lib.bra_gpu_pipe_records_bound.restype = C.c_uint64
    lib.bra_gpu_frame_chunks.argtypes = [vp, vp, vp, vp, C.c_uint32, vp, C.c_uint64, u64p, vp]
    lib.bra_gpu_frame_chunks.restype = C.c_int
    lib.bra_gpu_unframe_chunks.argtypes = [vp, vp, C.c_uint64, C.c_uint32, vp, vp, u32p, vp]
    lib.bra_gpu_unframe_chunks.restype = C.c_int
    lib.bra_gpu_compress_chunks.argtypes = [vp, vp, C.c_uint64, C.c_uint32, vp, C.c_uint64, u64p, u32p, vp]
    lib.bra_gpu_compress_chunks.restype = C.c_int
    lib.bra_gpu_decompress_chunks.argtypes = [vp, vp, C.c_uint64, C.c_uint32, vp, C.c_uint64, u64p, C.c_uint32, u32p, vp]
    lib.bra_gpu_decompress_chunks.restype = C.c_int
    lib.bra_gpu_host_alloc.argtypes = [vp, C.c_uint64]
    lib.bra_gpu_host_alloc.restype = vp
    lib.bra_gpu_host_free.argtypes = [vp, vp]
    lib.bra_gpu_host_free.restype = None
    lib.bra_gpu_compress_chunks_stage.argtypes = [vp, C.c_int, vp, C.c_uint64]
    lib.bra_gpu_compress_chunks_stage.restype = C.c_int
    lib.bra_gpu_compress_chunks_submit.argtypes = [vp, C.c_int, vp, C.c_uint64, C.c_uint32]
    lib.bra_gpu_compress_chunks_submit.restype = C.c_int
    lib.bra_gpu_compress_chunks_collect.argtypes = [vp, C.c_int, vp, C.c_uint64, u64p, u32p]
    lib.bra_gpu_compress_chunks_collect.restype = C.c_int
    lib.bra_gpu_chunks_crc32c_shard.argtypes = [vp, vp, C.c_uint64, C.c_uint32, vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_int,
                                                vp, vp]
    lib.bra_gpu_chunks_crc32c_shard.restype = C.c_int
    lib.bra_gpu_assemble_shards.argtypes = [vp, C.c_uint32, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), u32p, C.c_int, vp, vp, vp,
                                            C.c_uint64, vp]
    lib.bra_gpu_assemble_shards.restype = C.c_int
    return lib


lib = _load()
_libc = C.CDLL(None)
_libc.free.argtypes = [C.c_void_p]


def _buf(data: bytes):
    return (C.c_uint8 * max(1, len(data))).from_buffer_copy(data if data else b"\0")


def version() -> str:
    return lib.bra_gpu_version().decode()


def crc32c_combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """bra_crc32c_combine with a 64-bit length (host arithmetic of the product library)."""
    return lib.bra_gpu_crc32c_combine(crc_a, crc_b, len_b)


def entry_crc32c(me_crc: int, chunks_size: int, chunks_crc: int, data_size: int, block_size: int = MAX_CHUNK_SIZE) -> int:
    """me->crc32 after a compressed file (lib_bra_io_file_chunks.c:291-292)."""
    return lib.bra_gpu_entry_crc32c(me_crc, chunks_size, chunks_crc, data_size, block_size)


# ------------------------------------------------------------------------------------------------
# reference encoder interface (src/encoders/*.h), one block per call
# ------------------------------------------------------------------------------------------------
def bwt_encode(buf: bytes):
    """bra_bwt_encode2: returns (last column, primary index) or None on failure."""
    n = len(buf)
    out = (C.c_uint8 * max(1, n))()
    pi = C.c_uint32()
    if not lib.bra_bwt_encode2(_buf(buf), n, C.byref(pi), out):
        return None
    return bytes(out)[:n], pi.value


def bwt_decode(buf: bytes, primary_index: int) -> bytes:
    """bra_bwt_decode2."""
    n = len(buf)
    out = (C.c_uint8 * max(1, n))()
    lib.bra_bwt_decode2(_buf(buf), n, primary_index, None, out)
    return bytes(out)[:n]


def mtf_encode(buf: bytes):
    """bra_mtf_encode2: MTF positions, or None on failure."""
    out = (C.c_uint8 * max(1, len(buf)))()
    if not lib.bra_mtf_encode2(_buf(buf), len(buf), out):
        return None
    return bytes(out)[: len(buf)]


def mtf_decode(buf: bytes) -> bytes:
    """bra_mtf_decode2."""
    out = (C.c_uint8 * max(1, len(buf)))()
    lib.bra_mtf_decode2(_buf(buf), len(buf), out)
    return bytes(out)[: len(buf)]


def rle_encode(buf: bytes):
    """bra_rle_encode: PackBits stream, or None when the C function returns false."""
    p, s = C.c_void_p(), C.c_size_t()
    if not lib.bra_rle_encode(_buf(buf), len(buf), C.byref(p), C.byref(s)):
        return None
    out = C.string_at(p, s.value)
    _libc.free(p)
    return out


def rle_decode_compute_size(buf: bytes) -> int:
    """bra_rle_decode_compute_size: 0 on a malformed or empty stream."""
    return lib.bra_rle_decode_compute_size(_buf(buf), len(buf))


def rle_decode(buf: bytes):
    """bra_rle_decode: decoded bytes, or None when the C function returns false."""
    p, s = C.c_void_p(), C.c_size_t()
    if not lib.bra_rle_decode(_buf(buf), len(buf), C.byref(p), C.byref(s)):
        return None
    out = C.string_at(p, s.value)
    _libc.free(p)
    return out


def huffman_encode(buf: bytes):
    """bra_huffman_encode: HuffmanChunk, or None (e.g. for an empty buffer)."""
    ch = lib.bra_huffman_encode(_buf(buf), len(buf))
    if not ch:
        return None
    m = ch.contents.meta
    data = C.string_at(ch.contents.data, m.encoded_size) if m.encoded_size else b""
    res = HuffmanChunk(bytes(m.lengths), m.orig_size, m.encoded_size, data)
    lib.bra_huffman_chunk_free(ch)
    return res


def huffman_decode(lengths: bytes, orig_size: int, encoded_size: int, data: bytes):
    """bra_huffman_decode: decoded bytes, or None when the reference would reject the stream."""
    meta = HuffmanMeta()
    C.memmove(meta.lengths, lengths, 256)
    meta.orig_size, meta.encoded_size = orig_size, encoded_size
    osz = C.c_uint32()
    p = lib.bra_huffman_decode(C.byref(meta), _buf(data), C.byref(osz))
    if not p:
        return None
    out = C.string_at(p, osz.value)
    _libc.free(p)
    return out


# ------------------------------------------------------------------------------------------------
# batched device-resident codec
# ------------------------------------------------------------------------------------------------
class BlockCodec:
    """Batched encode/decode of independent blocks resident in HBM (torch uint8 CUDA tensors)."""

    def __init__(self, device: int = 0):
        self.device = device
        self.ctx = lib.bra_gpu_ctx_create(device)
        if not self.ctx:
            raise RuntimeError("bra_gpu_ctx_create failed (no usable MI355X?)")

    def close(self):
        if self.ctx:
            lib.bra_gpu_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def num_blocks(total: int, block_size: int) -> int:
        return lib.bra_gpu_num_blocks(total, block_size)

    @staticmethod
    def payload_bound(total: int, block_size: int) -> int:
        return lib.bra_gpu_payload_bound(total, block_size)

    def encode(self, data, block_size: int, headers=None, offsets=None, payload=None, stream=None):
        """Encode a uint8 CUDA tensor; returns (headers[nb,268] u8, offsets[nb+1] i64, payload u8)."""
        import torch

        total = data.numel()
        nb = self.num_blocks(total, block_size)
        dev = data.device
        if headers is None:
            headers = torch.empty((nb, HEADER_BYTES), dtype=torch.uint8, device=dev)
        if offsets is None:
            offsets = torch.empty((nb + 1,), dtype=torch.int64, device=dev)
        if payload is None:
            payload = torch.empty((int(total * 1.25) + 64 * nb + 4096,), dtype=torch.uint8, device=dev)
        s = _stream_handle(stream)
        rc = lib.bra_gpu_encode_blocks(self.ctx, data.data_ptr(), total, block_size, headers.data_ptr(), offsets.data_ptr(),
                                       payload.data_ptr(), payload.numel(), s)
        if rc == -2:
            need = int(offsets[nb].item())
            payload = torch.empty((need + 4096,), dtype=torch.uint8, device=dev)
            rc = lib.bra_gpu_encode_blocks(self.ctx, data.data_ptr(), total, block_size, headers.data_ptr(), offsets.data_ptr(),
                                           payload.data_ptr(), payload.numel(), s)
        if rc != 0:
            raise RuntimeError(f"bra_gpu_encode_blocks failed ({rc})")
        return headers, offsets, payload

    def decode(self, headers, offsets, payload, total: int, block_size: int, out=None, stream=None):
        import torch

        if out is None:
            out = torch.empty((total,), dtype=torch.uint8, device=headers.device)
        s = _stream_handle(stream)
        rc = lib.bra_gpu_decode_blocks(self.ctx, headers.data_ptr(), offsets.data_ptr(), payload.data_ptr(), total, block_size,
                                       out.data_ptr(), s)
        if rc != 0:
            raise RuntimeError(f"bra_gpu_decode_blocks failed ({rc})")
        return out

    # ---- the .BRa chunk stream (rows f1/f2) ----
    def crc32c(self, data, prev: int = 0, stream=None) -> int:
        """bra_crc32c(data, len, prev) of a uint8 CUDA tensor, computed on the device."""
        import torch

        out = torch.empty((1,), dtype=torch.int32, device=data.device)
        s = _stream_handle(stream)
        if lib.bra_gpu_crc32c(self.ctx, data.data_ptr(), data.numel(), prev, out.data_ptr(), s) != 0:
            raise RuntimeError("bra_gpu_crc32c failed")
        return int(out.item()) & 0xFFFFFFFF

    def chunks_crc32c(self, data, headers, block_size: int, prev: int = 0, stream=None) -> int:
        """CRC32C of hdr0||chunk0||hdr1||... (the compress loop's crc32 for prev=0)."""
        import torch

        out = torch.empty((1,), dtype=torch.int32, device=data.device)
        s = _stream_handle(stream)
        if lib.bra_gpu_chunks_crc32c(self.ctx, data.data_ptr(), data.numel(), block_size, headers.data_ptr(), prev, out.data_ptr(), s) != 0:
            raise RuntimeError("bra_gpu_chunks_crc32c failed")
        return int(out.item()) & 0xFFFFFFFF

    def frame(self, headers, offsets, payload, out=None, stream=None):
        """The chunk records of an encode() result, back to back (uint8 CUDA tensor)."""
        import torch

        nb = headers.shape[0]
        need = int(offsets[nb].item()) + 267 * nb
        if out is None:
            out = torch.empty((max(need, 1),), dtype=torch.uint8, device=headers.device)
        size = C.c_uint64()
        s = _stream_handle(stream)
        rc = lib.bra_gpu_frame_chunks(self.ctx, headers.data_ptr(), offsets.data_ptr(), payload.data_ptr(), nb, out.data_ptr(), out.numel(),
                                      C.byref(size), s)
        if rc != 0:
            raise RuntimeError(f"bra_gpu_frame_chunks failed ({rc})")
        return out[: size.value]

    def unframe(self, stream_t, max_chunks: int | None = None, stream=None):
        """(headers [n,268] u8, payload offsets [n+1] i64) of a chunk stream; raises on a malformed one."""
        import torch

        size = stream_t.numel()
        cap = max_chunks if max_chunks is not None else size // 268 + 1
        hdr = torch.empty((max(cap, 1), HEADER_BYTES), dtype=torch.uint8, device=stream_t.device)
        off = torch.empty((cap + 1,), dtype=torch.int64, device=stream_t.device)
        n = C.c_uint32()
        s = _stream_handle(stream)
        rc = lib.bra_gpu_unframe_chunks(self.ctx, stream_t.data_ptr(), size, cap, hdr.data_ptr(), off.data_ptr(), C.byref(n), s)
        if rc != 0:
            raise ValueError(f"bra_gpu_unframe_chunks rejected the stream ({rc}, {n.value} records)")
        return hdr[: n.value], off[: n.value]

    def compress_chunks(self, data, block_size: int = MAX_CHUNK_SIZE, out=None, stream=None):
        """The reference compress loop on the device: (chunk stream tensor, crc32, compressed?)."""
        import torch

        total = data.numel()
        cap = lib.bra_gpu_chunks_bound(total, block_size)
        if out is None or out.numel() < cap:
            out = torch.empty((cap,), dtype=torch.uint8, device=data.device)
        size, crc = C.c_uint64(), C.c_uint32()
        s = _stream_handle(stream)
        rc = lib.bra_gpu_compress_chunks(self.ctx, data.data_ptr(), total, block_size, out.data_ptr(), out.numel(), C.byref(size), C.byref(crc), s)
        if rc < 0:
            raise RuntimeError(f"bra_gpu_compress_chunks failed ({rc})")
        return out[: size.value], crc.value, rc == 1

    def compress_chunks_pipelined(self, data_np, batch_bytes: int, block_size: int = MAX_CHUNK_SIZE, stage_ahead: bool = True):
        """Host-buffer compression in batches with two in flight (bra_gpu_compress_chunks_stage /
        _submit / _collect, the front end's loop): [(records bytes, batch crc, compressed?)] per batch.
        stage_ahead: batch k + 1's input copy is queued before batch k is submitted (else submit
        makes each batch's copy itself)."""
        total = int(data_np.size)
        bb = max(block_size, batch_bytes // block_size * block_size)
        spans = [(o, min(total, o + bb)) for o in range(0, total, bb)]
        cap = lib.bra_gpu_pipe_records_bound(bb, block_size)
        hin = [lib.bra_gpu_host_alloc(self.ctx, bb) for _ in range(2)]
        hout = lib.bra_gpu_host_alloc(self.ctx, cap)
        if not all(hin) or not hout:
            raise RuntimeError("bra_gpu_host_alloc failed")
        res = []
        try:
            def fill(k):
                lo, hi = spans[k]
                C.memmove(hin[k % 2], data_np[lo:hi].ctypes.data, hi - lo)

            def stage(k):
                lo, hi = spans[k]
                fill(k)
                if lib.bra_gpu_compress_chunks_stage(self.ctx, k % 2, hin[k % 2], hi - lo) != 0:
                    raise RuntimeError("bra_gpu_compress_chunks_stage failed")

            def submit(k):
                lo, hi = spans[k]
                if lib.bra_gpu_compress_chunks_submit(self.ctx, k % 2, hin[k % 2], hi - lo, block_size) != 0:
                    raise RuntimeError("bra_gpu_compress_chunks_submit failed")

            def collect(k):
                size, crc = C.c_uint64(), C.c_uint32()
                rc = lib.bra_gpu_compress_chunks_collect(self.ctx, k % 2, hout, cap, C.byref(size), C.byref(crc))
                if rc < 0:
                    raise RuntimeError(f"bra_gpu_compress_chunks_collect failed ({rc})")
                res.append((C.string_at(hout, size.value), crc.value, rc == 1))

            if stage_ahead:
                stage(0)
                for k in range(len(spans)):
                    if k + 1 < len(spans):
                        stage(k + 1)  # slot (k + 1) % 2: batch k - 1 there is submitted, its input consumed on the device first
                    submit(k)
                    if k:
                        collect(k - 1)
                collect(len(spans) - 1)
            else:
                fill(0)
                submit(0)
                for k in range(len(spans)):
                    if k + 1 < len(spans):
                        fill(k + 1)
                        submit(k + 1)
                    collect(k)
        finally:
            # after a failure part way a slot may still hold a submitted batch or a staged copy:
            # drain both (a no-op on a free slot) so later pipelined calls find them free
            for q in range(2):
                lib.bra_gpu_compress_chunks_collect(self.ctx, q, None, 0, None, None)
            for p in (*hin, hout):
                lib.bra_gpu_host_free(self.ctx, p)
        return res

    def decompress_chunks(self, stream_t, block_size: int = MAX_CHUNK_SIZE, out_cap: int | None = None, prev_crc: int = 0, stream=None):
        """The reference decode loop on the device: (decoded tensor, crc chained from prev_crc)."""
        import torch

        size = stream_t.numel()
        if out_cap is None:
            out_cap = (size // 268 + 1) * block_size
        out = torch.empty((max(out_cap, 1),), dtype=torch.uint8, device=stream_t.device)
        osz, crc = C.c_uint64(), C.c_uint32()
        s = _stream_handle(stream)
        rc = lib.bra_gpu_decompress_chunks(self.ctx, stream_t.data_ptr(), size, block_size, out.data_ptr(), out_cap, C.byref(osz), prev_crc,
                                           C.byref(crc), s)
        if rc != 0:
            raise ValueError(f"bra_gpu_decompress_chunks rejected the stream ({rc})")
        return out[: osz.value], crc.value

    # ---- sharded streams (row e) ----
    def chunks_crc32c_shard(self, data, headers, block_size: int, first_chunk: int, chunk_stride: int, global_total: int,
                            with_init: bool, out=None, prev: int = 0, stream=None):
        """This shard's CRC word (int32 CUDA tensor [1]) of the global chunk stream; XOR over the shards
        gives the stream's CRC32C when exactly one shard has with_init.  Asynchronous on `stream`."""
        import torch

        if out is None:
            out = torch.empty((1,), dtype=torch.int32, device=data.device)
        s = _stream_handle(stream)
        rc = lib.bra_gpu_chunks_crc32c_shard(self.ctx, data.data_ptr(), data.numel(), block_size, headers.data_ptr(), first_chunk,
                                             chunk_stride, global_total, prev, 1 if with_init else 0, out.data_ptr(), s)
        if rc != 0:
            raise RuntimeError(f"bra_gpu_chunks_crc32c_shard failed ({rc})")
        return out

    def assemble_shards(self, parts, round_robin: bool = True, headers=None, offsets=None, payload=None, stream=None):
        """parts: [(headers [n_p,268] u8, offsets [n_p+1] i64, payload u8)] on this device.  Returns
        (headers, offsets, payload) of all blocks in global order (round robin: block g from part g % P)."""
        import torch

        P = len(parts)
        nbs = [int(h.shape[0]) for h, _, _ in parts]
        nb = sum(nbs)
        dev = parts[0][0].device
        total_pay = sum(int(p.numel()) for _, _, p in parts)
        if headers is None:
            headers = torch.empty((nb, HEADER_BYTES), dtype=torch.uint8, device=dev)
        if offsets is None:
            offsets = torch.empty((nb + 1,), dtype=torch.int64, device=dev)
        given = payload is not None
        if payload is None:  # the parts' payload capacities: the assembly cannot overflow it
            payload = torch.empty((max(total_pay, 1),), dtype=torch.uint8, device=dev)
        arr = C.c_void_p * P
        hp = arr(*[h.data_ptr() for h, _, _ in parts])
        op = arr(*[o.data_ptr() for _, o, _ in parts])
        pp = arr(*[p.data_ptr() for _, _, p in parts])
        nn = (C.c_uint32 * P)(*nbs)
        s = _stream_handle(stream)
        rc = lib.bra_gpu_assemble_shards(self.ctx, P, hp, op, pp, nn, 1 if round_robin else 0, headers.data_ptr(), offsets.data_ptr(),
                                         payload.data_ptr(), payload.numel(), s)
        if rc != 0:
            raise RuntimeError(f"bra_gpu_assemble_shards failed ({rc})")
        if given and int(offsets[nb].item()) == -1:  # the asynchronous call's overflow marker
            raise RuntimeError("bra_gpu_assemble_shards: payload capacity too small")
        return headers, offsets, payload

    def prof_enable(self, mask: int):
        """Time the selected kernel slots with HIP events (bit i = slot i, see csrc/prof.h)."""
        lib.bra_gpu_prof_enable(self.ctx, mask)

    def prof_reset(self):
        lib.bra_gpu_prof_reset(self.ctx)

    def prof_read(self) -> dict:
        """{slot name: (total device ms, launches, algorithmic bytes)} since the last reset."""
        out = {}
        n = lib.bra_gpu_prof_read(self.ctx, -1, None, None, None, None)
        for i in range(n):
            name, ms, cnt, by = C.c_char_p(), C.c_double(), C.c_uint32(), C.c_double()
            lib.bra_gpu_prof_read(self.ctx, i, C.byref(name), C.byref(ms), C.byref(cnt), C.byref(by))
            out[name.value.decode()] = (ms.value, cnt.value, by.value)
        return out

    SLOTS = ("stage.bwt", "stage.mtf", "stage.rle", "stage.huffman",
             "bwt.l0_hist", "bwt.l0_scatter", "bwt.pack", "bwt.hist", "bwt.scan", "bwt.scatter", "bwt.jobs", "bwt.mjobs", "bwt.fallback",
             "mtf.lastocc", "mtf.scan", "mtf.encode",
             "rle.runs", "rle.link", "rle.sizes", "rle.offsets", "rle.write",
             "huf.build", "huf.offsets", "huf.tilebits", "huf.tilescan", "huf.zero", "huf.pack",
             "chunks.frame", "chunks.crc",
             "dec.huffman", "dec.rle", "dec.mtf", "dec.ibwt",
             "dec.hd_trans", "dec.rled", "dec.mtf_local", "dec.ib_walk", "dec.ib_pair")
    DECODE_KERNELS = ("dec.hd_trans", "dec.rled", "dec.mtf_local", "dec.ib_walk")

    @classmethod
    def slot_mask(cls, *names) -> int:
        m = 0
        for n in names:
            m |= 1 << cls.SLOTS.index(n)
        return m

    def debug_rerun_jobs(self, reps: int, shuffle_seed: int = 0) -> int:
        """Re-run the last encode's BWT job phase `reps` times (job inputs reordered when
        shuffle_seed != 0), auditing each run: the failing jobs summed over the runs."""
        f = lib.bra_gpu_debug_rerun_jobs
        f.argtypes, f.restype = [C.c_void_p, C.c_int, C.c_uint], C.c_int
        r = f(self.ctx, reps, shuffle_seed)
        if r < 0:
            raise RuntimeError("bra_gpu_debug_rerun_jobs failed")
        return r

    def stage_ptr(self, stage: int) -> int:
        return lib.bra_gpu_stage_ptr(self.ctx, stage) or 0

    def stage_copy(self, stage: int, nbytes: int):
        """Host copy (numpy uint8) of the first `nbytes` of an intermediate stage of the last encode."""
        import numpy as np
        import torch

        torch.cuda.synchronize()
        out = np.empty(nbytes, np.uint8)
        hip = C.CDLL("libamdhip64.so")
        rc = hip.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(self.stage_ptr(stage)), C.c_size_t(nbytes), 2)  # D2H
        if rc != 0:
            raise RuntimeError(f"hipMemcpy failed ({rc})")
        return out


def sortnet_selftest(waves: int, groups: int = 4096, iters: int = 64, seed: int = 1) -> int:
    """Failing sorts of the BWT job sort (bra_gpu_sortnet_selftest) on random key sets."""
    f = lib.bra_gpu_sortnet_selftest
    f.argtypes, f.restype = [C.c_int, C.c_uint, C.c_uint, C.c_uint, C.c_void_p], C.c_int
    r = f(waves, groups, iters, seed, None)
    if r < 0:
        raise RuntimeError("bra_gpu_sortnet_selftest failed")
    return r


def _stream_handle(stream):
    """The HIP stream a call runs on: the given torch stream, else torch's current stream -- so that
    a call without a stream is ordered with the torch work around it (allocations, copies, reads of
    the results); the context's own stream is not, and a caller reading a result tensor on torch's
    stream could see it before the call's last kernels had written it."""
    import torch

    return (stream if stream is not None else torch.cuda.current_stream()).cuda_stream


def parse_header(h: bytes):
    """(primary_index, lengths, orig_size, encoded_size) of a 268-byte in-memory chunk header."""
    pi = int.from_bytes(h[0:4], "little")
    return pi, bytes(h[4:260]), int.from_bytes(h[260:264], "little"), int.from_bytes(h[264:268], "little")


# ------------------------------------------------------------------------------------------------
# synthetic inputs (csrc/bra_synth.c)
# ------------------------------------------------------------------------------------------------
_synth = None


def synth_lib():
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise ImportError(f"{SYNTH_PATH} not built")
        _synth = C.CDLL(SYNTH_PATH)
        _synth.bra_synth_block.argtypes = [C.c_int, C.c_uint64, C.c_void_p, C.c_uint64]
        _synth.bra_synth_fill.argtypes = [C.c_int, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint64]
        _synth.bra_synth_fill_strided.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint64]
    return _synth


def synth_block(kind: int, index: int, n: int) -> bytes:
    b = (C.c_uint8 * max(1, n))()
    synth_lib().bra_synth_block(kind, index, b, n)
    return bytes(b)[:n]


def synth_fill(kind: int, total: int, block_size: int, first_block: int = 0, stride: int = 1):
    """numpy uint8 array of `total` bytes: synthetic blocks first_block, first_block + stride, ..."""
    import numpy as np

    a = np.empty(total, dtype=np.uint8)
    synth_lib().bra_synth_fill_strided(kind, first_block, stride, a.ctypes.data, total, block_size)
    return a
