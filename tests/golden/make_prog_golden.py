"""Generate tests/golden/prog.json: archives made by the REFERENCE programs (src/prog).

Run in the build container (where /root/reference exists):
    make -C oracle ref gpulib progs && python tests/golden/make_prog_golden.py

oracle/_ref/prog_cpu/{bra,unbra} are the reference's own programs compiled from its unchanged
sources and linked against the reference lib_bra (CPU encoders).  Every case below is run in a
fresh directory laid out by `stage_inputs`; the fixture stores the size and sha256 of the .BRa the
reference `bra` writes, and the `unbra -l` listing (stdout), so that tests/test_gpu_prog.py can run
the SAME programs linked against lib_bra on libbra_hip.so (prog_gpu) and compare the archive bytes.
The flows follow test/test_bra.cpp:332-398 (bra -c, unbra -l, unbra -t, unbra -y -o <dir>).
Data only (sizes, digests, listings), no code.
"""
from __future__ import annotations

import hashlib
import importlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

# name -> (bra arguments after `bra -c -o <name>.BRa`)
CASES = {
    "lorem": ["fixtures/lorem.txt"],                      # test_bra_unbra_comp_2 (test_bra.cpp:353-371)
    "text_3MiB": ["big/text_3MiB.txt"],                   # 13 chunks of 256 KiB, the last ragged
    "mixed_dir": ["-r", "mixed"],                         # a directory: text, sym16, random (stored), lorem
}


def stage_inputs(d: str) -> None:
    """The input tree every case runs in (deterministic synthetic data, csrc/bra_synth.c)."""
    bra = importlib.import_module("br-archive_amd")
    os.makedirs(os.path.join(d, "fixtures"))
    os.makedirs(os.path.join(d, "big"))
    os.makedirs(os.path.join(d, "mixed", "sub"))
    shutil.copy(os.path.join(ROOT, "tests", "golden", "lorem.txt"), os.path.join(d, "fixtures", "lorem.txt"))
    shutil.copy(os.path.join(ROOT, "tests", "golden", "lorem.txt"), os.path.join(d, "mixed", "sub", "lorem.txt"))
    files = {
        "big/text_3MiB.txt": (bra.SYNTH_TEXT, 3 * 1048576 + 12345, 0),
        "mixed/a_text.txt": (bra.SYNTH_TEXT, 700000, 7),
        "mixed/b_sym16.bin": (bra.SYNTH_SYM16, 600000, 3),
        "mixed/c_random.bin": (bra.SYNTH_RANDOM, 300000, 5),
    }
    for rel, (kind, n, first) in files.items():
        with open(os.path.join(d, rel), "wb") as f:
            f.write(bra.synth_fill(kind, n, 262144, first_block=first).tobytes())


def run(prog_dir: str, cwd: str, *args: str) -> subprocess.CompletedProcess:
    return subprocess.run([os.path.join(prog_dir, args[0]), *args[1:]], cwd=cwd, capture_output=True, text=True, timeout=600)


def make_archive(prog_dir: str, d: str, name: str, args: list[str]) -> bytes:
    r = run(prog_dir, d, "bra", "-y", "-c", "-o", f"{name}.BRa", *args)
    if r.returncode != 0:
        raise RuntimeError(f"bra {name}: {r.returncode} {r.stdout[-500:]} {r.stderr[-500:]}")
    return open(os.path.join(d, f"{name}.BRa"), "rb").read()


def main():
    cpu = os.path.join(ROOT, "oracle", "_ref", "prog_cpu")
    if not os.path.exists(os.path.join(cpu, "bra")):
        sys.exit("oracle/_ref/prog_cpu missing: run `make -C oracle progs` where /root/reference exists")
    out = {}
    with tempfile.TemporaryDirectory() as d:
        stage_inputs(d)
        for name, args in CASES.items():
            a = make_archive(cpu, d, name, args)
            lst = run(cpu, d, "unbra", "-l", f"{name}.BRa")
            assert lst.returncode == 0, lst.stdout
            out[name] = {"args": args, "size": len(a), "sha256": hashlib.sha256(a).hexdigest(), "list_stdout": lst.stdout}
            print(name, len(a), out[name]["sha256"], flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "prog.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
