"""The drop-in boundary: libbra_hip.so loads and exports exactly the C-ABI of include/bra_hip.h.

CPU-only: no function that touches the GPU is called here.
"""
import importlib
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bra_hip.h")


def _header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bra_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_exports_header_symbols():
    bra = importlib.import_module("br-archive_amd")
    out = subprocess.check_output(["nm", "-D", "--defined-only", bra.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    declared = _header_functions()
    assert len(declared) == 47
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert sorted(bra.ABI_SYMBOLS) == declared
    # the reference's 14 encoder entry points are all there
    ref14 = [f for f in declared if not f.startswith("bra_gpu_")]
    assert len(ref14) == 14


def test_library_does_not_define_reference_logger():
    # lib_bra keeps bra_log_*; the codec only references bra_log_error weakly
    bra = importlib.import_module("br-archive_amd")
    out = subprocess.check_output(["nm", "-D", bra.LIB_PATH], text=True)
    defined = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert not any(s.startswith("bra_log") for s in defined)
    weak = [l for l in out.splitlines() if l.endswith(" bra_log_error")]
    assert weak and weak[0].split()[-2] in ("w", "v")


def test_host_only_helpers():
    bra = importlib.import_module("br-archive_amd")
    assert bra.version().startswith("bra_hip")
    assert bra.BlockCodec.num_blocks(256 << 20, 1 << 20) == 256
    assert bra.BlockCodec.num_blocks((256 << 20) + 1, 1 << 20) == 257
    assert bra.BlockCodec.payload_bound(1 << 20, 1 << 20) >= 4 * (1 << 20)


def test_synthetic_generators_deterministic():
    bra = importlib.import_module("br-archive_amd")
    a = bra.synth_block(bra.SYNTH_TEXT, 5, 4096)
    assert a == bra.synth_block(bra.SYNTH_TEXT, 5, 4096)
    assert a != bra.synth_block(bra.SYNTH_TEXT, 6, 4096)
    assert set(bra.synth_block(bra.SYNTH_SYM16, 0, 4096)) <= set(range(ord("a"), ord("a") + 16))
    assert bra.synth_block(bra.SYNTH_TILED, 0, 38) == b"Test File Fixture.\n" * 2


def _undefined_bra(path):
    import subprocess

    out = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.split()[-1].startswith("bra_")}


def _defined(path):
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines()}


@pytest.mark.parametrize("lib", ["libbralib_hipenc.so", "libbralib_gpu.so"])
def test_lib_bra_links_against_gpu_library(lib):
    """lib_bra built from the reference sources minus src/encoders (oracle/Makefile target gpulib,
    linked with -Wl,--no-undefined): every bra_* symbol it needs from outside is exported by
    libbra_hip.so, and it carries no encoder of its own."""
    path = os.path.join(ROOT, "oracle", "_ref", lib)
    if not os.path.exists(path):
        pytest.skip(f"{lib} not built (needs the reference tree)")
    hip = os.path.join(ROOT, "br-archive_amd", "libbra_hip.so")
    need = _undefined_bra(path)
    assert need and need <= _defined(hip), need - _defined(hip)
    encoders = {"bra_bwt_encode2", "bra_mtf_encode2", "bra_rle_encode", "bra_huffman_encode", "bra_huffman_decode"}
    assert not (encoders & _defined(path))
    if lib == "libbralib_hipenc.so":  # the reference's own chunk loop calls the drop-in encoders
        assert {"bra_bwt_encode2", "bra_mtf_encode2", "bra_rle_encode", "bra_huffman_encode", "bra_huffman_chunk_free"} <= need
    else:  # the batched front end calls the batch ABI
        assert {"bra_gpu_compress_chunks_stage", "bra_gpu_compress_chunks_submit", "bra_gpu_compress_chunks_collect", "bra_gpu_decompress_chunks_host"} <= need


def test_pipe_records_bound_covers_every_chunk():
    """bra_gpu_pipe_records_bound (host arithmetic, no device): at least the on-disk record of every
    chunk at its RLE capacity (n + ceil(n / 128) + 16 payload bytes + 267 header bytes) and at most
    about 1.01x the batch plus the headers."""
    bra = importlib.import_module("br-archive_amd")
    lib = bra.lib
    cs = bra.MAX_CHUNK_SIZE
    for total in (1, 100, cs - 1, cs, cs + 1, 3 * cs + 7, 256 * cs):
        b = lib.bra_gpu_pipe_records_bound(total, cs)
        need, o = 0, 0
        while o < total:
            n = min(cs, total - o)
            need += n + (n + 127) // 128 + 16 + 267
            o += n
        assert need <= b <= need + 4096 + 64 * (total // cs + 1)
    assert lib.bra_gpu_pipe_records_bound(0, cs) == 0
