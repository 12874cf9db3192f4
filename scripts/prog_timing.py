"""Wall-clock timing of the reference's own programs (src/prog `bra -c` / `unbra`) linked against
the GPU library (oracle/_ref/prog_gpu) and against the reference lib_bra (oracle/_ref/prog_cpu),
on a synthetic text file.  Measurement only.

    python scripts/prog_timing.py [gpu_mib] [cpu_mib] [outdir] [nmany]

The GPU programs compress and extract a gpu_mib file (default 1024); the CPU programs a cpu_mib one
(default 64: the reference encodes ~2.3 MB/s on one core, so 1 GiB would take ~8 minutes) -- both
are bytes / wall seconds of the whole program run (file I/O included).  Each archive is extracted
again and compared with its input; the two programs' archives of the cpu_mib prefix are compared
byte for byte.  The GPU runs also report the front end's own per-file breakdown (BRA_FRONT_TIMING),
the fixed cost of a run on a 4 KiB file, and an archive of nmany (default 128) 8 MiB files.
Prints one JSON line.
"""
import hashlib
import importlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


FRONT = []  # the front end's per-file breakdown lines (BRA_FRONT_TIMING=1) of the last run


def run(prog, cwd, *args):
    env = dict(os.environ, BRA_FRONT_TIMING="1")
    t0 = time.perf_counter()
    r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", prog), *args], cwd=cwd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=1100,
                       env=env)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"{prog} {args} rc {r.returncode}: {r.stderr[-500:]!r}")
    FRONT[:] = [ln for ln in r.stderr.decode(errors="replace").splitlines() if ln.startswith("front:")]
    return dt


def main():
    gpu_mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    cpu_mib = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    out = sys.argv[3] if len(sys.argv) > 3 else "/tmp/prog_timing"
    nmany = int(sys.argv[4]) if len(sys.argv) > 4 else 128
    bra = importlib.import_module("br-archive_amd")
    os.makedirs(out, exist_ok=True)
    res = {"file": "synthetic text (BASELINE configs[1] generator, 1 MiB blocks concatenated)", "chunk_bytes": 256 * 1024}
    for tag, mib, progs in (("gpu", gpu_mib, "prog_gpu"), ("cpu", cpu_mib, "prog_cpu")):
        d = os.path.join(out, tag)
        os.makedirs(os.path.join(d, "x"), exist_ok=True)
        name = f"text_{mib}MiB.txt"
        src = os.path.join(d, name)
        bra.synth_fill(bra.SYNTH_TEXT, mib << 20, 1 << 20).tofile(src)
        for p in (os.path.join(d, "a.BRa"),):
            if os.path.exists(p):
                os.remove(p)
        tc = run(f"{progs}/bra", d, "-y", "-c", "-o", "a.BRa", name)
        front_c = list(FRONT)
        tx = run(f"{progs}/unbra", d, "-y", "-o", "x", "a.BRa")
        front_x = list(FRONT)
        same = sha(src) == sha(os.path.join(d, "x", name))
        if tag == "cpu":
            # the GPU programs on the same file: the archive must be the reference's, byte for byte
            run("prog_gpu/bra", d, "-y", "-c", "-o", "g.BRa", name)
            res["archives_identical_on_cpu_file"] = sha(os.path.join(d, "g.BRa")) == sha(os.path.join(d, "a.BRa"))
        res[tag] = {"bytes": mib << 20, "archive_bytes": os.path.getsize(os.path.join(d, "a.BRa")), "compress_s": round(tc, 3),
                    "compress_GBps": round((mib << 20) / tc / 1e9, 5), "extract_s": round(tx, 3), "extract_GBps": round((mib << 20) / tx / 1e9, 5),
                    "roundtrip_identical": same, "archive_sha256": sha(os.path.join(d, "a.BRa"))}
        if tag == "gpu":
            res[tag]["front_compress"] = front_c
            res[tag]["front_extract"] = front_x
            # fixed cost of a run: the same program on a 4 KiB file (process start, HIP runtime and
            # context creation, exit)
            tiny = os.path.join(d, "tiny.txt")
            bra.synth_fill(bra.SYNTH_TEXT, 4096, 4096).tofile(tiny)
            res[tag]["tiny_4KiB_compress_s"] = round(min(run(f"{progs}/bra", d, "-y", "-c", "-o", "t.BRa", "tiny.txt") for _ in range(3)), 3)
            res[tag]["tiny_front"] = list(FRONT)
            # many medium files in one archive (pinned buffers reused across files)
            many = os.path.join(d, "many")
            os.makedirs(many, exist_ok=True)
            names = []
            for i in range(nmany):
                fn = os.path.join(many, f"f{i:03d}.txt")
                bra.synth_fill(bra.SYNTH_TEXT, 8 << 20, 1 << 20, first_block=1000 + 8 * i).tofile(fn)
                names.append(os.path.join("many", f"f{i:03d}.txt"))
            tm = run(f"{progs}/bra", d, "-y", "-c", "-o", "m.BRa", *names)
            res[tag]["many_files"] = {"files": nmany, "file_bytes": 8 << 20, "compress_s": round(tm, 3),
                                      "compress_GBps": round(nmany * (8 << 20) / tm / 1e9, 5), "archive_bytes": os.path.getsize(os.path.join(d, "m.BRa"))}
        print(json.dumps({tag: res[tag]}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
