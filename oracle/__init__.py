"""oracle -- TEST INFRASTRUCTURE ONLY.

ctypes bindings to
  * ``liboracle.so``        -- the CPU restatement of the reference chain (``bra_oracle.c``);
  * ``_ref/libbraref.so``   -- the reference's own ``src/encoders`` compiled from /root/reference
                               by ``oracle/Makefile`` (absent when the reference tree was never
                               available; then only the restatement + committed golden vectors);
  * ``_ref/libbralib.so``   -- the whole reference ``lib_bra`` plus ``oracle/ref_chunks.c``, a
                               driver of its chunk loop (``bra_io_file_chunks_compress_file``)
                               and CRC32C, for the chunk-stream and framing parity (rows f1/f2).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
package, and only as the checker.  The product library (``br-archive_amd/``) never links it.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
# BRA_ORACLE_DIR: load liboracle.so / libbraref.so / libbralib.so from another build of them (the
# host-sanitizer build, oracle/_ref/asan, `make -C oracle asan`; tests/test_asan.py)
_ALT = os.environ.get("BRA_ORACLE_DIR")
_libc = C.CDLL(None)
_libc.free.argtypes = [C.c_void_p]


class HuffMeta(C.Structure):
    """Packed bra_huffman_t (src/lib_bra_types.h:51-56)."""

    _pack_ = 1
    _fields_ = [("lengths", C.c_uint8 * 256), ("orig_size", C.c_uint32), ("encoded_size", C.c_uint32)]


assert C.sizeof(HuffMeta) == 264


@dataclass
class Chunk:
    """One encoded block: what bra_io_file_chunks_compress_file writes (pi + meta + payload)."""

    primary_index: int
    bwt: bytes
    mtf: bytes
    rle: bytes
    lengths: bytes
    orig_size: int
    encoded_size: int
    payload: bytes

    def header_bytes(self) -> bytes:
        """The 267-byte on-disk chunk header (lib_bra_io_file_chunks.c:76-95)."""
        return (
            self.primary_index.to_bytes(4, "little")[:3]
            + self.lengths
            + self.orig_size.to_bytes(4, "little")
            + self.encoded_size.to_bytes(4, "little")
        )


def _buf(data: bytes):
    return (C.c_uint8 * max(1, len(data))).from_buffer_copy(data if data else b"\0")


# --------------------------------------------------------------------------------------------
# CPU restatement
# --------------------------------------------------------------------------------------------
class Oracle:
    """The restatement (bra_oracle.c).  Method names follow the reference encoder API."""

    def __init__(self, path: str | None = None):
        path = path or os.path.join(_ALT or _HERE, "liboracle.so")
        self.lib = L = C.CDLL(path)
        u8p, u32p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32)
        L.orc_bwt_encode.argtypes = [u8p, C.c_uint32, u32p, u8p, u32p]
        L.orc_bwt_decode.argtypes = [u8p, C.c_uint32, C.c_uint32, u8p]
        L.orc_mtf_encode.argtypes = [u8p, C.c_size_t, u8p]
        L.orc_mtf_decode.argtypes = [u8p, C.c_size_t, u8p]
        L.orc_rle_encode.argtypes = [u8p, C.c_size_t, u8p]
        L.orc_rle_encode.restype = C.c_size_t
        L.orc_rle_decode_size.argtypes = [u8p, C.c_size_t]
        L.orc_rle_decode_size.restype = C.c_size_t
        L.orc_rle_decode.argtypes = [u8p, C.c_size_t, u8p]
        L.orc_rle_decode.restype = C.c_size_t
        L.orc_huffman_encode.argtypes = [u8p, C.c_uint32, C.POINTER(HuffMeta), C.POINTER(C.c_void_p)]
        L.orc_huffman_decode.argtypes = [C.POINTER(HuffMeta), u8p, u8p]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_crc32c.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32]
        L.orc_crc32c.restype = C.c_uint32
        L.orc_crc32c_combine.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_crc32c_combine.restype = C.c_uint32
        L.orc_chunks_crc32c.argtypes = [u8p, u8p, C.c_uint64, C.c_uint32, C.c_uint32]
        L.orc_chunks_crc32c.restype = C.c_uint32
        L.orc_entry_crc32c.argtypes = [C.c_uint32, C.c_int64, C.c_uint32, C.c_uint64]
        L.orc_entry_crc32c.restype = C.c_uint32
        L.orc_frame_record.argtypes = [u8p, u8p, C.c_uint32, u8p]
        L.orc_frame_record.restype = C.c_size_t

    def bwt_encode(self, data: bytes, want_sa: bool = False):
        n = len(data)
        out = (C.c_uint8 * n)()
        pi = C.c_uint32()
        sa = (C.c_uint32 * n)() if want_sa else None
        ok = self.lib.orc_bwt_encode(_buf(data), n, C.byref(pi), out, sa)
        if not ok:
            raise ValueError("bwt_encode failed")
        if want_sa:
            return bytes(out), pi.value, list(sa)
        return bytes(out), pi.value

    def bwt_decode(self, data: bytes, pi: int) -> bytes:
        n = len(data)
        out = (C.c_uint8 * n)()
        if not self.lib.orc_bwt_decode(_buf(data), n, pi, out):
            raise ValueError("bwt_decode failed")
        return bytes(out)

    def mtf_encode(self, data: bytes) -> bytes:
        out = (C.c_uint8 * len(data))()
        if not self.lib.orc_mtf_encode(_buf(data), len(data), out):
            raise ValueError("mtf_encode failed")
        return bytes(out)

    def mtf_decode(self, data: bytes) -> bytes:
        out = (C.c_uint8 * len(data))()
        if not self.lib.orc_mtf_decode(_buf(data), len(data), out):
            raise ValueError("mtf_decode failed")
        return bytes(out)

    def rle_encode(self, data: bytes) -> bytes:
        n = self.lib.orc_rle_encode(_buf(data), len(data), None)
        out = (C.c_uint8 * max(1, n))()
        self.lib.orc_rle_encode(_buf(data), len(data), out)
        return bytes(out)[:n]

    def rle_decode_compute_size(self, data: bytes) -> int:
        return self.lib.orc_rle_decode_size(_buf(data), len(data))

    def rle_decode(self, data: bytes):
        s = self.rle_decode_compute_size(data)
        if s == 0:
            return None
        out = (C.c_uint8 * s)()
        self.lib.orc_rle_decode(_buf(data), len(data), out)
        return bytes(out)

    def huffman_encode(self, data: bytes):
        meta = HuffMeta()
        p = C.c_void_p()
        if not self.lib.orc_huffman_encode(_buf(data), len(data), C.byref(meta), C.byref(p)):
            return None
        payload = C.string_at(p, meta.encoded_size)
        self.lib.orc_free(p)
        return bytes(meta.lengths), meta.orig_size, meta.encoded_size, payload

    def huffman_decode(self, lengths: bytes, orig_size: int, encoded_size: int, payload: bytes):
        meta = HuffMeta()
        C.memmove(meta.lengths, lengths, 256)
        meta.orig_size, meta.encoded_size = orig_size, encoded_size
        out = (C.c_uint8 * max(1, orig_size))()
        if not self.lib.orc_huffman_decode(C.byref(meta), _buf(payload), out):
            return None
        return bytes(out)[:orig_size]

    def encode_block(self, data: bytes) -> Chunk:
        b, pi = self.bwt_encode(data)
        m = self.mtf_encode(b)
        r = self.rle_encode(m)
        lens, osz, esz, pay = self.huffman_encode(r)
        return Chunk(pi, b, m, r, lens, osz, esz, pay)

    def decode_block(self, ch: Chunk) -> bytes:
        r = self.huffman_decode(ch.lengths, ch.orig_size, ch.encoded_size, ch.payload)
        m = self.rle_decode(r)
        b = self.mtf_decode(m)
        return self.bwt_decode(b, ch.primary_index)

    # ---- CRC32C and the chunk stream (rows f1/f2) ----
    def crc32c(self, data: bytes, prev: int = 0) -> int:
        return self.lib.orc_crc32c(_buf(data), len(data), prev)

    def crc32c_combine(self, a: int, b: int, len_b: int) -> int:
        return self.lib.orc_crc32c_combine(a, b, len_b & 0xFFFFFFFF)

    def chunks_crc32c(self, headers: bytes, data: bytes, chunk_size: int, prev: int = 0) -> int:
        """crc32 of the compress loop (lib_bra_io_file_chunks.c:248-249): headers = n x 268 B."""
        return self.lib.orc_chunks_crc32c(_buf(headers), _buf(data), len(data), chunk_size, prev)

    def entry_crc32c(self, me_crc: int, tmpfile_size: int, chunks_crc: int, data_size: int) -> int:
        """me->crc32 after a compressed file (lib_bra_io_file_chunks.c:291-292)."""
        return self.lib.orc_entry_crc32c(me_crc, tmpfile_size, chunks_crc, data_size)

    def frame(self, chunks: list) -> bytes:
        """The tmpfile of the compress loop: every chunk as 3-B pi + 264-B meta + payload."""
        out = []
        for ch in chunks:
            rec = (C.c_uint8 * (267 + ch.encoded_size))()
            hdr = ch.primary_index.to_bytes(4, "little") + ch.lengths + ch.orig_size.to_bytes(4, "little") + ch.encoded_size.to_bytes(4, "little")
            n = self.lib.orc_frame_record(_buf(hdr), _buf(ch.payload), ch.encoded_size, rec)
            out.append(bytes(rec)[:n])
        return b"".join(out)

    def compress_chunks(self, data: bytes, chunk_size: int = 256 * 1024):
        """(tmpfile bytes, crc32, chunks) as bra_io_file_chunks_compress_file builds them."""
        chunks = [self.encode_block(data[i : i + chunk_size]) for i in range(0, len(data), chunk_size)]
        hdrs = b"".join(ch.primary_index.to_bytes(4, "little") + ch.lengths + ch.orig_size.to_bytes(4, "little") + ch.encoded_size.to_bytes(4, "little") for ch in chunks)
        return self.frame(chunks), self.chunks_crc32c(hdrs, data, chunk_size), chunks


# --------------------------------------------------------------------------------------------
# Reference encoders compiled from /root/reference (oracle/_ref/libbraref.so)
# --------------------------------------------------------------------------------------------
REF_PATH = os.path.join(_ALT or os.path.join(_HERE, "_ref"), "libbraref.so")


def have_ref() -> bool:
    return os.path.exists(REF_PATH)


class Reference:
    """The reference's own src/encoders, called through its C-ABI (bra_*.h)."""

    def __init__(self, path: str = REF_PATH):
        self.lib = L = C.CDLL(path)
        u8p, u32p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32)
        L.bra_bwt_encode2.argtypes = [u8p, C.c_uint32, u32p, u8p]
        L.bra_bwt_encode2.restype = C.c_bool
        L.bra_bwt_decode2.argtypes = [u8p, C.c_uint32, C.c_uint32, u32p, u8p]
        L.bra_mtf_encode2.argtypes = [u8p, C.c_size_t, u8p]
        L.bra_mtf_encode2.restype = C.c_bool
        L.bra_mtf_decode2.argtypes = [u8p, C.c_size_t, u8p]
        L.bra_rle_encode.argtypes = [u8p, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        L.bra_rle_encode.restype = C.c_bool
        L.bra_rle_decode.argtypes = [u8p, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        L.bra_rle_decode.restype = C.c_bool
        L.bra_rle_decode_compute_size.argtypes = [u8p, C.c_size_t]
        L.bra_rle_decode_compute_size.restype = C.c_size_t
        L.bra_huffman_encode.argtypes = [u8p, C.c_uint32]
        L.bra_huffman_encode.restype = C.c_void_p
        L.bra_huffman_decode.argtypes = [C.POINTER(HuffMeta), u8p, u32p]
        L.bra_huffman_decode.restype = C.c_void_p
        L.bra_huffman_chunk_free.argtypes = [C.c_void_p]

    def bwt_encode(self, data: bytes):
        n = len(data)
        out = (C.c_uint8 * n)()
        pi = C.c_uint32()
        if not self.lib.bra_bwt_encode2(_buf(data), n, C.byref(pi), out):
            raise ValueError("bra_bwt_encode2 failed")
        return bytes(out), pi.value

    def bwt_decode(self, data: bytes, pi: int) -> bytes:
        n = len(data)
        out = (C.c_uint8 * n)()
        tr = (C.c_uint32 * n)()
        self.lib.bra_bwt_decode2(_buf(data), n, pi, tr, out)
        return bytes(out)

    def mtf_encode(self, data: bytes) -> bytes:
        out = (C.c_uint8 * len(data))()
        self.lib.bra_mtf_encode2(_buf(data), len(data), out)
        return bytes(out)

    def mtf_decode(self, data: bytes) -> bytes:
        out = (C.c_uint8 * len(data))()
        self.lib.bra_mtf_decode2(_buf(data), len(data), out)
        return bytes(out)

    def rle_encode(self, data: bytes) -> bytes:
        p, s = C.c_void_p(), C.c_size_t()
        if not self.lib.bra_rle_encode(_buf(data), len(data), C.byref(p), C.byref(s)):
            raise ValueError("bra_rle_encode failed")
        out = C.string_at(p, s.value)
        _libc.free(p)
        return out

    def rle_decode_compute_size(self, data: bytes) -> int:
        return self.lib.bra_rle_decode_compute_size(_buf(data), len(data))

    def rle_decode(self, data: bytes):
        p, s = C.c_void_p(), C.c_size_t()
        if not self.lib.bra_rle_decode(_buf(data), len(data), C.byref(p), C.byref(s)):
            return None
        out = C.string_at(p, s.value)
        _libc.free(p)
        return out

    def huffman_encode(self, data: bytes):
        p = self.lib.bra_huffman_encode(_buf(data), len(data))
        if not p:
            return None
        meta = HuffMeta.from_address(p)
        lens, osz, esz = bytes(meta.lengths), meta.orig_size, meta.encoded_size
        dptr = C.c_void_p.from_address(p + 264).value
        payload = C.string_at(dptr, esz) if esz else b""
        self.lib.bra_huffman_chunk_free(p)
        return lens, osz, esz, payload

    def huffman_decode(self, lengths: bytes, orig_size: int, encoded_size: int, payload: bytes):
        meta = HuffMeta()
        C.memmove(meta.lengths, lengths, 256)
        meta.orig_size, meta.encoded_size = orig_size, encoded_size
        osz = C.c_uint32()
        p = self.lib.bra_huffman_decode(C.byref(meta), _buf(payload), C.byref(osz))
        if not p:
            return None
        out = C.string_at(p, osz.value)
        _libc.free(p)
        return out

    def encode_block(self, data: bytes) -> Chunk:
        b, pi = self.bwt_encode(data)
        m = self.mtf_encode(b)
        r = self.rle_encode(m)
        lens, osz, esz, pay = self.huffman_encode(r)
        return Chunk(pi, b, m, r, lens, osz, esz, pay)

    def decode_block(self, ch: Chunk) -> bytes:
        r = self.huffman_decode(ch.lengths, ch.orig_size, ch.encoded_size, ch.payload)
        m = self.rle_decode(r)
        b = self.mtf_decode(m)
        return self.bwt_decode(b, ch.primary_index)


# --------------------------------------------------------------------------------------------
# The whole reference lib_bra (oracle/_ref/libbralib.so): CRC32C and the chunk loop
# --------------------------------------------------------------------------------------------
LIB_PATH = os.path.join(_ALT or os.path.join(_HERE, "_ref"), "libbralib.so")


def have_reflib() -> bool:
    return os.path.exists(LIB_PATH)


class ReferenceLib:
    """bra_crc32c / bra_crc32c_combine (lib_bra_crc32c.h) and the reference chunk loop driven by
    oracle/ref_chunks.c on real files."""

    def __init__(self, path: str = LIB_PATH):
        self.lib = L = C.CDLL(path)
        L.bra_crc32c.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32]
        L.bra_crc32c.restype = C.c_uint32
        L.bra_crc32c_combine.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.bra_crc32c_combine.restype = C.c_uint32
        L.ref_compress_file.argtypes = [C.c_char_p, C.c_char_p, C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.ref_compress_file.restype = C.c_int
        L.ref_decompress_file.argtypes = [C.c_char_p, C.c_char_p, C.c_uint64, C.POINTER(C.c_uint32)]
        L.ref_decompress_file.restype = C.c_int

    def crc32c(self, data: bytes, prev: int = 0) -> int:
        return self.lib.bra_crc32c(_buf(data), len(data), prev)

    def crc32c_combine(self, a: int, b: int, len_b: int) -> int:
        return self.lib.bra_crc32c_combine(a, b, len_b & 0xFFFFFFFF)

    def compress_file(self, data: bytes, workdir: str):
        """Run bra_io_file_chunks_compress_file on `data`.  Returns (ok, dst bytes, me->crc32
        before, me->crc32 after, attributes after).  dst holds the meta entry (when compressed)
        followed by the chunk records."""
        src = os.path.join(workdir, "src.bin")
        dst = os.path.join(workdir, "dst.bin")
        with open(src, "wb") as f:
            f.write(data)
        cb, ca, at = C.c_uint32(), C.c_uint32(), C.c_uint32()
        ok = self.lib.ref_compress_file(src.encode(), dst.encode(), len(data), C.byref(cb), C.byref(ca), C.byref(at))
        with open(dst, "rb") as f:
            out = f.read()
        return bool(ok), out, cb.value, ca.value, at.value

    def decompress_file(self, stream: bytes, workdir: str):
        """Run bra_io_file_chunks_decompress_file on chunk records.  Returns (ok, decoded bytes,
        me->crc32 after)."""
        src = os.path.join(workdir, "stream.bin")
        dst = os.path.join(workdir, "decoded.bin")
        with open(src, "wb") as f:
            f.write(stream)
        crc = C.c_uint32()
        ok = self.lib.ref_decompress_file(src.encode(), dst.encode(), len(stream), C.byref(crc))
        out = open(dst, "rb").read() if os.path.exists(dst) else b""
        return bool(ok), out, crc.value
