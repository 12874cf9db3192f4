"""The reference's programs on the GPU library (SURVEY 8.1 row b: "src/prog links unchanged").

oracle/_ref/prog_gpu/{bra,unbra,bra.sfx} are compiled from the reference's UNCHANGED src/prog
sources (oracle/Makefile target `progs`) and linked with -Wl,--no-undefined against
oracle/_ref/libbralib_gpu.so: lib_bra whose encoders and chunk loop are libbra_hip.so and the
batched front end (br-archive_amd/frontend/bra_io_file_chunks_gpu.c).  The same programs linked
against the reference lib_bra (prog_cpu) made tests/golden/prog.json (make_prog_golden.py).

The flows are the reference's own (test/test_bra.cpp:332-398): `bra -c -o x.BRa <inputs>`, then
`unbra -l`, `unbra -t` and `unbra -y -o <dir>`; plus the self-extracting archive (`bra -s`, then
running the .brx).  Bar: the GPU-made archive is byte-identical to the reference's, its listing
is the reference's, and every extracted file equals its input.
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from make_prog_golden import CASES, stage_inputs  # noqa: E402

GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "prog.json")))
PROG = os.path.join(ROOT, "oracle", "_ref", "prog_gpu")
REF_DIR = os.path.join(ROOT, "oracle", "_ref")


def _run(cwd, exe, *args, env=None):
    return subprocess.run([exe, *args], cwd=cwd, capture_output=True, text=True, timeout=300, env=env)


def _tree(d):
    out = {}
    for base, _, files in os.walk(d):
        for f in files:
            p = os.path.join(base, f)
            out[os.path.relpath(p, d)] = hashlib.sha256(open(p, "rb").read()).hexdigest()
    return out


def test_programs_linked_against_gpu_library():
    """The three programs exist and resolve lib_bra and the HIP library (no GPU call)."""
    for exe in ("bra", "unbra", "bra.sfx"):
        p = os.path.join(PROG, exe)
        assert os.path.exists(p), f"{p} not built (make -C oracle progs where the reference tree exists)"
        r = subprocess.run(["ldd", p], capture_output=True, text=True)
        assert "not found" not in r.stdout, r.stdout
        assert "libbralib_gpu.so" in r.stdout and "libbra_hip.so" in r.stdout, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_bra_unbra_on_gpu_matches_reference(name, tmp_path):
    d = str(tmp_path / "work")
    os.makedirs(d)
    stage_inputs(d)
    g = GOLDEN[name]
    r = _run(d, os.path.join(PROG, "bra"), "-y", "-c", "-o", f"{name}.BRa", *g["args"])
    assert r.returncode == 0, r.stdout[-1000:] + r.stderr[-1000:]
    a = open(os.path.join(d, f"{name}.BRa"), "rb").read()
    assert (len(a), hashlib.sha256(a).hexdigest()) == (g["size"], g["sha256"]), "archive differs from the reference's"
    r = _run(d, os.path.join(PROG, "unbra"), "-l", f"{name}.BRa")
    assert r.returncode == 0 and r.stdout == g["list_stdout"], r.stdout[-2000:]
    r = _run(d, os.path.join(PROG, "unbra"), "-t", f"{name}.BRa")
    assert r.returncode == 0, r.stdout[-1000:] + r.stderr[-1000:]
    r = _run(d, os.path.join(PROG, "unbra"), "-y", "-o", "out", f"{name}.BRa")
    assert r.returncode == 0, r.stdout[-1000:] + r.stderr[-1000:]
    src, got = _tree(d), _tree(os.path.join(d, "out"))
    assert got, "nothing extracted"
    for rel, h in got.items():
        assert src[rel] == h, rel


@pytest.mark.gpu
def test_self_extracting_archive_on_gpu(tmp_path):
    d = str(tmp_path / "work")
    os.makedirs(d)
    stage_inputs(d)
    shutil.copy(os.path.join(PROG, "bra.sfx"), os.path.join(d, "bra.sfx"))  # bra looks for it in the cwd (BRA_SFX_FILENAME)
    r = _run(d, os.path.join(PROG, "bra"), "-y", "-c", "-s", "-o", "text_sfx", "big/text_3MiB.txt", "fixtures/lorem.txt")
    assert r.returncode == 0, r.stdout[-1000:] + r.stderr[-1000:]
    x = str(tmp_path / "extract")
    os.makedirs(x)
    shutil.copy(os.path.join(d, "text_sfx.BRa.brx"), os.path.join(x, "text_sfx.BRa.brx"))
    env = dict(os.environ, LD_LIBRARY_PATH=REF_DIR + os.pathsep + os.environ.get("LD_LIBRARY_PATH", ""))
    r = _run(x, os.path.join(x, "text_sfx.BRa.brx"), "-y", env=env)
    assert r.returncode == 0, r.stdout[-1000:] + r.stderr[-1000:]
    src = _tree(d)
    for rel in ("big/text_3MiB.txt", "fixtures/lorem.txt"):
        assert _tree(x).get(rel) == src[rel], rel
