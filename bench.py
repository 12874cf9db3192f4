#!/usr/bin/env python3
"""bench.py -- br-archive block codec on MI355X: encode GB/s of input bytes (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic blocks already resident in HBM:
every block goes through BWT -> MTF -> PackBits RLE -> canonical Huffman (the chunk encoder of
lib_bra_io_file_chunks.c:217-245), the chunk-stream CRC32C is computed (:248-249) and the compressed
chunks are assembled in global block order on rank 0 (SURVEY 8.1 rows d, e, f2).

Sharding (SURVEY 8.1 row e, BASELINE configs[3]): global block b is encoded by rank b mod G (round
robin); with G > 1 the compressed chunks and CRC shares are gathered to rank 0 over RCCL/xGMI inside
the step.  Weak scaling (default): every rank holds --bytes-per-gpu (256 MiB = configs[1] per GPU; at
G = 8 this is configs[3]'s 2 GiB).  Strong scaling: --total-bytes fixes the global input (2 GiB for
configs[3] at any G); a rank then encodes its share in batches of at most --batch-bytes.

`python bench.py --gpus N` with N > 1 and no torchrun environment starts torchrun itself (a child
process launched before anything touches the GPU) and relays its output and exit code.

Printed (rank 0, one JSON line): the metric, `roofline` for the dominant kernel (algorithmic bytes per
launch / average launch time measured with HIP events on the codec's stream during the timed steps),
and `cpu_baseline`: the reference's own src/encoders (oracle/_ref/libbraref.so, compiled from the
reference sources) timed on this host, single-threaded and on all the cores this box gives us.
"""
import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "encode GB/s (input bytes) on 256 MiB synthetic blocks, 1/2/4/8 GPU; bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
KINDS = {"text": 0, "random": 1, "sym16": 2, "tiled": 3}
# the BASELINE.json config each input kind is quoted on
WORKLOADS = {
    "text": "BASELINE configs[1]: 1 MiB enwik-style synthetic text blocks (Zipf word stream)",
    "random": "BASELINE configs[2]: uniform-random bytes",
    "sym16": "BASELINE configs[4]: 16-symbol geometric low-entropy blocks",
    "tiled": "BASELINE configs[0] input: test/test.txt (19 B) tiled",
}
CPU_SHARE = 16  # host CPUs per GPU on the box (os.cpu_count() reports the whole machine)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--kind", default="text", choices=sorted(KINDS))
    ap.add_argument("--block-size", type=int, default=1 << 20)
    ap.add_argument("--bytes-per-gpu", type=int, default=256 << 20, help="weak scaling: input bytes per rank")
    ap.add_argument("--total-bytes", type=int, default=0, help="strong scaling: global input bytes (e.g. 2147483648)")
    ap.add_argument("--batch-bytes", type=int, default=256 << 20, help="largest batch one encode call takes")
    ap.add_argument("--cpu-threads", type=int, default=CPU_SHARE)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--profile-all", action="store_true", help="time every kernel during the timed steps")
    ap.add_argument("--no-secondary", action="store_true", help="skip the decode and PCIe-inclusive measurements")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--gather-mode", default="exact", choices=["exact", "bound"],
                    help="N > 1: payloads gathered at their exact sizes (one size all_gather per step) or at the geometry's bound")
    ap.add_argument("--pcie-batches", type=int, default=4, help="batches of the split transfer-inclusive encode (two contexts)")
    ap.add_argument("--pcie-stream", type=int, default=4, help="batches of the streamed transfer-inclusive encode (pipelined API)")
    return ap.parse_args()


def spawn_torchrun(args) -> int:
    """Relaunch this script under torchrun with one rank per GPU; no GPU call has happened yet."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_sample_sizes(nb, bs, threads):
    """Blocks timed single-threaded (about 4 MiB) and on `threads` workers (about 2 MiB per thread):
    10-30 s of reference CPU work for 1 MiB text or random blocks."""
    return max(1, min(nb, (4 << 20) // bs)), max(1, min(nb, threads * max(1, (2 << 20) // bs)))


def cgroup_cpu_max() -> str:
    """The cgroup v2 CPU quota of this process ("max 100000" = unlimited), or "unknown"."""
    try:
        return open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        return "unknown"


def cpu_baseline(data_np, bs, threads, gpu_chunks, all_host_cores=True):
    """The reference encoders on host cores (one block per task; ctypes drops the GIL), on a bounded
    sample of the benchmark's own blocks: single-threaded, then `threads` workers (skipped when the
    sample is one block, e.g. configs[0]'s single 64 KiB block)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import Oracle, Reference, have_ref

    impl, kind = (Reference(), "reference") if have_ref() else (Oracle(), "port")
    n1, nm = cpu_sample_sizes(data_np.size // bs, bs, threads)
    blocks = [data_np[i * bs:(i + 1) * bs].tobytes() for i in range(max(n1, nm))]
    t0 = time.perf_counter()
    one = [impl.encode_block(b) for b in blocks[:n1]]
    dt1 = time.perf_counter() - t0
    if nm > 1:
        threads = max(1, min(threads, nm))
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            many = list(ex.map(impl.encode_block, blocks[:nm]))
        dtm = time.perf_counter() - t0
    else:
        threads, many, dtm = 1, one, dt1
    chunks = many if nm >= n1 else one
    same = all((c.primary_index, c.lengths, c.orig_size, c.encoded_size, c.payload) == g for c, g in zip(chunks, gpu_chunks))
    all_cores = None
    if nm > 1 and all_host_cores:
        # every host CPU this process may run on ("1-thread and all-host-cores"):
        # one block per worker, as many blocks as workers (bounded by the batch)
        na = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
        na_blocks = max(1, min(data_np.size // bs, na))
        ins = blocks + [data_np[i * bs:(i + 1) * bs].tobytes() for i in range(len(blocks), na_blocks)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(min(na, na_blocks)) as ex:
            res_all = list(ex.map(impl.encode_block, ins[:na_blocks]))
        dta = time.perf_counter() - t0
        ok_all = all((c.primary_index, c.lengths, c.orig_size, c.encoded_size, c.payload) ==
                     (d.primary_index, d.lengths, d.orig_size, d.encoded_size, d.payload) for c, d in zip(res_all, chunks))
        all_cores = {"value": round(na_blocks * bs / dta / 1e9, 6), "unit": "GB/s", "cores": min(na, na_blocks), "nproc": os.cpu_count(),
                     "affinity_cpus": na, "cgroup_cpu_max": cgroup_cpu_max(),
                     "sample": f"{na_blocks} x {bs} B blocks, one block per task on {min(na, na_blocks)} threads ({dta:.2f} s wall)",
                     "same_output_as_16_thread_run": bool(ok_all)}
        quota = cgroup_cpu_max().split()
        if len(quota) == 2 and quota[0].isdigit() and quota[1].isdigit() and int(quota[1]):
            cpus = int(quota[0]) / int(quota[1])
            all_cores["note"] = (f"the cgroup quota caps this process at {cpus:g} CPUs, so {min(na, na_blocks)} threads share {cpus:g} CPUs: "
                                 f"the {threads}-thread figure above is this host's real ceiling for the reference encoder")
    return {
        "value": round(nm * bs / dtm / 1e9, 6),
        "unit": "GB/s",
        "cores": threads,
        "kind": kind,
        "sample": f"{nm} x {bs} B blocks of the benchmark input, one block per task on {threads} threads ({dtm:.2f} s wall); "
                  f"{cpu_model()}, {os.cpu_count()} host CPUs visible, {CPU_SHARE} per GPU on this box",
        "single_thread": {"value": round(n1 * bs / dt1 / 1e9, 6), "unit": "GB/s", "cores": 1,
                          "sample": f"{n1} x {bs} B blocks, {dt1:.2f} s", "seconds_per_block": round(dt1 / n1, 4)},
        "bit_exact_vs_gpu": bool(same),
        "blocks_checked": len(chunks),
        "all_cores": all_cores,
    }


def block_digest(pi, lens, osz, esz, payload) -> str:
    """sha256(pi u32 LE || bra_huffman_t || payload): the per-block digest of tests/golden/digests.json."""
    import hashlib

    h = hashlib.sha256()
    h.update(pi.to_bytes(4, "little") + lens + osz.to_bytes(4, "little") + esz.to_bytes(4, "little") + payload)
    return h.hexdigest()


def reference_digests(kind, bs, nbg):
    """Per-global-block reference digests for this workload from tests/golden/digests.json (made
    from the reference's own encoders by tests/golden/make_digests.py), or None when no workload
    there covers blocks 0..nbg-1 of this kind and block size."""
    path = os.path.join(ROOT, "tests", "golden", "digests.json")
    if not os.path.exists(path):
        return None
    best = None
    for w in json.load(open(path)).values():
        if (w["kind"], w["block_size"], w["first_block"], w["stride"]) == (KINDS[kind], bs, 0, 1) and w["nblocks"] >= nbg:
            if best is None or w["nblocks"] < best["nblocks"]:
                best = w
    return best


def check_vs_reference(H, O, P, kind, bs, nbg, global_total, world, threads):
    """Rank 0's check of the ASSEMBLED global stream (every rank's blocks) against the reference:
    every block against the committed reference digests when they cover the workload, and a
    sample of blocks spread over the global range (all ranks' shards) re-encoded live by the
    reference encoders (oracle/_ref) on this host."""
    import numpy as np

    bra = importlib.import_module("br-archive_amd")
    hdr_h, off_h, pay_h = H.cpu().numpy(), O.cpu().numpy(), P.cpu().numpy()

    def chunk(b):
        pi, lens, osz, esz = bra.parse_header(hdr_h[b].tobytes())
        return pi, lens, osz, esz, pay_h[off_h[b]:off_h[b] + esz].tobytes()

    res = {}
    w = reference_digests(kind, bs, nbg)
    if w is not None and global_total == nbg * bs:
        bad = [b for b in range(nbg) if block_digest(*chunk(b)) != w["sha256"][b]]
        res["digests"] = {"blocks": nbg, "mismatches": len(bad), "bit_exact": not bad, "first_bad": bad[:4],
                          "source": "tests/golden/digests.json (reference src/encoders, every block)"}
    if world > 1:
        from concurrent.futures import ThreadPoolExecutor

        from oracle import Oracle, Reference, have_ref

        impl = Reference() if have_ref() else Oracle()
        sample = sorted({int(x) for x in np.linspace(0, nbg - 1, num=min(nbg, 2 * world))})
        ins = [bra.synth_block(KINDS[kind], b, min(bs, global_total - b * bs)) for b in sample]
        with ThreadPoolExecutor(max(1, threads)) as ex:
            refs = list(ex.map(impl.encode_block, ins))
        same = all((c.primary_index, c.lengths, c.orig_size, c.encoded_size, c.payload) == chunk(b) for c, b in zip(refs, sample))
        res["live"] = {"blocks": sample, "bit_exact": bool(same), "ranks": sorted({b % world for b in sample}),
                       "source": "oracle/_ref/libbraref.so" if have_ref() else "oracle port"}
    return res


def pcie_inclusive(codec, data_np, d, bs, nb, hdr, off, pay, payload_bytes, work_stream, nbatch, codec2=None, split=None):
    """Transfer-inclusive encode (SURVEY 8.1(d) secondary): pinned host input -> HBM, encode, chunk
    headers + payload back to pinned host memory, timed from the first byte sent to the last byte
    received.  Serial: one copy in, one encode, the copies out, on one stream.  Overlapped: the
    input in `nbatch` batches, every host-to-device copy queued at once on a copy stream, and two
    contexts (codec, codec2) on two streams and two host threads encoding alternate batches (batch
    k waits for its copy's event), so one batch's kernels run while another's input arrives and
    while the other context's host thread follows its own level loop; each batch's payload goes
    back on a copy stream as soon as its thread has read its size.  (One context encoding the
    batches one after the other paid each call's fixed cost -- 4.3 ms per 64 MiB batch against
    12.8 ms per 256 MiB -- and ran slower than the serial form.)"""
    import threading

    import torch

    total = data_np.size
    h_in = torch.from_numpy(data_np).pin_memory()
    h_hdr = torch.empty(hdr.shape, dtype=torch.uint8).pin_memory()
    h_pay = torch.empty((payload_bytes + 4096 * (nbatch + 1),), dtype=torch.uint8).pin_memory()
    res = {}
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(2):
        with torch.cuda.stream(work_stream):
            d.copy_(h_in, non_blocking=True)
            codec.encode(d, bs, hdr, off, pay, stream=work_stream)
            h_hdr.copy_(hdr, non_blocking=True)
            h_pay[:payload_bytes].copy_(pay[:payload_bytes], non_blocking=True)
    torch.cuda.synchronize()
    res["encode_pcie_inclusive_serial_GBps"] = round(2 * total / (time.perf_counter() - t1) / 1e9, 4)
    if codec2 is None:
        return res
    # overlapped: batches of whole blocks
    if split:  # batch sizes in blocks (the rest of the input, if any, is one more batch)
        cuts = [0]
        for c in split:
            cuts.append(min(nb, cuts[-1] + c))
        if cuts[-1] < nb:
            cuts.append(nb)
        parts = [(a, b) for a, b in zip(cuts, cuts[1:]) if b > a]
    else:
        per = max(1, -(-nb // nbatch))
        parts = [(b0, min(nb, b0 + per)) for b0 in range(0, nb, per)]
    # copy streams at high priority: HIP shares a few hardware queues among a process's streams of
    # one priority, and a kernel queued behind a copy's barrier on a shared queue waits for that
    # copy (batch k's encode then waited for batch k + 1's input; scripts/micro/ev_wait.py)
    h2d = torch.cuda.Stream(priority=-1)
    streams = [work_stream, torch.cuda.Stream()]
    d2hs = [torch.cuda.Stream(priority=-1), torch.cuda.Stream(priority=-1)]
    codecs = [codec, codec2]
    offs = [torch.empty((b1 - b0 + 1,), dtype=torch.int64, device=d.device) for b0, b1 in parts]
    # payload room per batch: a block's payload never exceeds its RLE bytes + 1 (an optimal prefix
    # code over byte symbols is never longer than the 8-bit code)
    cap = [(b1 - b0) * (bs + bs // 128 + 64) + 4096 for b0, b1 in parts]
    pbase = [sum(cap[:k]) for k in range(len(parts))]
    if pbase[-1] + cap[-1] > pay.numel():
        return res
    sizes = torch.empty((len(parts),), dtype=torch.int64).pin_memory()
    hb = [0] * (len(parts) + 1)

    def worker(t, ev_in, errs):
        try:
            for k in range(t, len(parts), 2):
                b0, b1 = parts[k]
                lo, hi = b0 * bs, min(total, b1 * bs)
                s = streams[t]
                s.wait_event(ev_in[k])
                with torch.cuda.stream(s):
                    codecs[t].encode(d[lo:hi], bs, hdr[b0:b1], offs[k], pay[pbase[k]:pbase[k] + cap[k]], stream=s)
                    sizes[k:k + 1].copy_(offs[k][-1:], non_blocking=True)
                    e = torch.cuda.Event()
                    e.record(s)
                e.synchronize()
                sz = int(sizes[k])
                hb[k + 1] = sz  # (the host offsets are prefix sums taken after the threads finish)
                d2h = d2hs[t]
                d2h.wait_event(e)
                with torch.cuda.stream(d2h):
                    h_hdr[b0:b1].copy_(hdr[b0:b1], non_blocking=True)
                    # each batch's payload lands at its own capacity offset of the host buffer
                    h_pay[pbase[k]:pbase[k] + sz].copy_(pay[pbase[k]:pbase[k] + sz], non_blocking=True)
                d2h.synchronize()
        except Exception as ex:  # reported by the caller
            errs.append(ex)

    if pbase[-1] + cap[-1] > h_pay.numel():
        h_pay = torch.empty((pbase[-1] + cap[-1],), dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    reps = 2
    for rep in range(reps + 1):  # rep 0 untimed: the second context's first encode allocates its workspace
        if rep == 1:
            torch.cuda.synchronize()
            t1 = time.perf_counter()
        ev_in = []
        with torch.cuda.stream(h2d):
            for b0, b1 in parts:
                lo, hi = b0 * bs, min(total, b1 * bs)
                d[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
                e = torch.cuda.Event()
                e.record(h2d)
                ev_in.append(e)
        errs = []
        th = [threading.Thread(target=worker, args=(t, ev_in, errs)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            raise errs[0]
    torch.cuda.synchronize()
    res["encode_pcie_inclusive_GBps"] = round(reps * total / (time.perf_counter() - t1) / 1e9, 4)
    res["encode_pcie_inclusive_batches"] = len(parts)
    res["encode_pcie_inclusive_contexts"] = 2
    res["encode_pcie_inclusive_bytes_back"] = int(sum(hb) + hdr.numel())
    return res


def copy_peak_GBps(dev, nbytes=512 << 20, reps=10):
    """A measured device copy-kernel peak (SURVEY 8.1 row d: report the fraction of it beside the
    spec peak): torch's copy kernel over nbytes, read + write bytes per second, HIP events."""
    import torch

    a = torch.empty((nbytes,), dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbps = 2.0 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbps


def pcie_stream(bra, codec, data_np, kind, bs, nstream):
    """Transfer-inclusive encode of a stream of host batches (SURVEY 8.1(d) secondary; the front
    end's loop): `nstream` batches of the configs[1] size go host -> HBM -> chunk records -> host
    through the library's pipelined API (bra_gpu_compress_chunks_stage / _submit / _collect, one
    context): batch k + 1's input copy is queued before batch k is submitted and batch k - 1's records
    come back while batch k's later stages run.  Timed from the first copy queued to the last record
    byte received; the input sits in pinned host memory (two distinct synthetic batches alternate).
    A batch's records are checked against the same batch's earlier records."""
    import ctypes as C

    lib = bra.lib
    total = data_np.size
    nb = -(-total // bs)
    second = bra.synth_fill(KINDS[kind], total, bs, first_block=nb)
    cap = lib.bra_gpu_chunks_bound(total, bs)
    hin = [lib.bra_gpu_host_alloc(codec.ctx, total) for _ in range(2)]
    hout = lib.bra_gpu_host_alloc(codec.ctx, cap)
    res = {}
    try:
        if not all(hin) or not hout:
            return res
        C.memmove(hin[0], data_np.ctypes.data, total)
        C.memmove(hin[1], second.ctypes.data, total)
        seen = {}

        def run(nbat):
            back = 0

            def collect(k):
                nonlocal back
                size, crc = C.c_uint64(), C.c_uint32()
                rc = lib.bra_gpu_compress_chunks_collect(codec.ctx, k % 2, hout, cap, C.byref(size), C.byref(crc))
                if rc < 0:
                    raise RuntimeError(f"bra_gpu_compress_chunks_collect failed ({rc})")
                back += size.value
                key = (size.value, crc.value, C.string_at(hout, min(size.value, 1 << 16)))
                if seen.setdefault(k % 2, key) != key:
                    raise RuntimeError("pipelined encode: the same batch gave different records")

            if lib.bra_gpu_compress_chunks_stage(codec.ctx, 0, hin[0], total) != 0:
                raise RuntimeError("bra_gpu_compress_chunks_stage failed")
            for k in range(nbat):
                if k + 1 < nbat and lib.bra_gpu_compress_chunks_stage(codec.ctx, (k + 1) % 2, hin[(k + 1) % 2], total) != 0:
                    raise RuntimeError("bra_gpu_compress_chunks_stage failed")
                if lib.bra_gpu_compress_chunks_submit(codec.ctx, k % 2, hin[k % 2], total, bs) != 0:
                    raise RuntimeError("bra_gpu_compress_chunks_submit failed")
                if k:
                    collect(k - 1)
            collect(nbat - 1)
            return back

        run(2)  # untimed: the pipeline's buffers are allocated
        t0 = time.perf_counter()
        back = run(nstream)
        dt = time.perf_counter() - t0
        res["encode_pcie_stream_GBps"] = round(nstream * total / dt / 1e9, 4)
        res["encode_pcie_stream"] = {"batches": nstream, "batch_bytes": int(total), "records_bytes_back": int(back), "contexts": 1}
    finally:
        for p in (*hin, hout):
            if p:
                lib.bra_gpu_host_free(codec.ctx, p)
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_torchrun(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist

    if args.backend != "nccl":
        # rehearsal of the N > 1 path on fewer devices (gloo: ranks may share a GPU); counting the
        # devices does not initialise the GPU
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))  # RCCL over xGMI
        else:
            dist.init_process_group(args.backend)
    bra = importlib.import_module("br-archive_amd")
    dmod = importlib.import_module("br-archive_amd.dist")

    bs = args.block_size
    strong = args.total_bytes > 0
    global_total = args.total_bytes if strong else world * args.bytes_per_gpu
    nbg = dmod.num_blocks(global_total, bs)
    my_blocks = dmod.shard_blocks(nbg, rank, world)
    my_bytes = dmod.shard_bytes(global_total, bs, rank, world)
    nb = len(my_blocks)
    data_np = bra.synth_fill(KINDS[args.kind], my_bytes, bs, first_block=rank, stride=world)
    d = torch.from_numpy(data_np).cuda()
    codec = bra.BlockCodec(local)
    dev = d.device
    def outputs():
        return (torch.empty((nb, bra.HEADER_BYTES), dtype=torch.uint8, device=dev), torch.empty((nb + 1,), dtype=torch.int64, device=dev),
                torch.empty((int(my_bytes * 1.25) + 64 * nb + 65536,), dtype=torch.uint8, device=dev),
                torch.zeros((1,), dtype=torch.int32, device=dev))

    # world > 1: two output sets, so that step i + 1 encodes while step i's chunks are gathered
    outs = [outputs() for _ in range(2 if world > 1 else 1)]
    hdr, off, pay, crc_share = outs[0]
    per_batch = max(1, args.batch_bytes // bs)
    batches = [(b0, min(nb, b0 + per_batch)) for b0 in range(0, nb, per_batch)]
    off_b = torch.empty((per_batch + 1,), dtype=torch.int64, device=dev)
    # exact sizes (default): one all_gather of (payload bytes, block count) per step, then each rank's
    # compressed bytes only.  The host waits for that all_gather, but the gather of step k is issued
    # after step k + 1's encode has been queued, so the GPU is never idle for it.  "bound": the sizes
    # follow from the geometry and the payloads travel at their bound (about 1.0x the shard's input
    # instead of its compressed size), no host wait.  (Unmeasured on hardware until a driver SCALE
    # record exists.)
    geo = (global_total, bs) if args.gather_mode == "bound" else None
    gather = dmod.ChunkGather(dist, rank, world, geometry=geo) if world > 1 else None
    work_stream = torch.cuda.Stream()
    gather_stream = torch.cuda.Stream() if world > 1 else None
    result = {}
    state = {"i": 0, "pending": None, "free": [None] * len(outs)}

    def gather_assemble(k, ev):
        """Gather output set k (its encode ended at event ev) to rank 0 and assemble it there, on the
        gather stream: the collectives wait for that encode only, not for the one queued after it, so
        the transfers run under the next step's kernels (the gather posts them at the geometry's
        payload bounds, with no host read of the gathered sizes)."""
        with torch.cuda.stream(gather_stream):
            gather_stream.wait_event(ev)
            parts = gather(*outs[k])
            if rank == 0:
                result["stream"] = dmod.assemble(codec, parts, round_robin=True, stream=gather_stream)
                result["crc_t"] = dmod.merge_crc_device(parts)
            e = torch.cuda.Event()
            e.record(gather_stream)
            state["free"][k] = e  # the set's sends are done: the next encode into it may start

    def flush():
        if state["pending"] is not None:
            gather_assemble(*state["pending"])
            state["pending"] = None

    def step():
        """Encode this rank's blocks and its CRC share; rank 0 assembles the chunks in global order.
        World > 1: the gather of this step's output to rank 0 is issued after the next step's encode
        has been queued (flush() issues the last one), so no rank waits on the host for the others."""
        k = state["i"] % len(outs)
        state["i"] += 1
        hdr, off, pay, crc_share = outs[k]
        if state["free"][k] is not None:
            work_stream.wait_event(state["free"][k])
        with torch.cuda.stream(work_stream):
            if len(batches) == 1:
                codec.encode(d, bs, hdr, off, pay, stream=work_stream)
            else:
                base = 0
                for b0, b1 in batches:
                    lo, hi = b0 * bs, min(my_bytes, b1 * bs)
                    codec.encode(d[lo:hi], bs, hdr[b0:b1], off_b, pay[base:], stream=work_stream)
                    off[b0:b1 + 1] = off_b[: b1 - b0 + 1] + base
                    base += int(off_b[b1 - b0].item())
            codec.chunks_crc32c_shard(d, hdr, bs, rank, world, global_total, rank == 0, out=crc_share, stream=work_stream)
            if world == 1:
                # assembled on the stream and the CRC merged on the device: a step has no host wait of
                # its own, so the host queues the next step while this one runs
                parts = [(hdr, off, pay, crc_share)]  # the payload's capacity: no host read of its size
                result["stream"] = dmod.assemble(codec, parts, round_robin=True)
                result["crc_t"] = dmod.merge_crc_device(parts)
                return
            ev = torch.cuda.Event()
            ev.record(work_stream)
        prev, state["pending"] = state["pending"], (k, ev)
        if prev is not None:
            gather_assemble(*prev)

    # ---- find the dominant kernel (one untimed, fully profiled pass) ----
    kernel_slots = [s for s in codec.SLOTS if not s.startswith(("stage.", "dec."))]
    enc_slots = [s for s in codec.SLOTS if not s.startswith("dec.")]
    codec.prof_enable(codec.slot_mask(*enc_slots))
    step()
    flush()
    torch.cuda.synchronize()
    prof0 = codec.prof_read()
    kernel_slots = [s for s in kernel_slots if s in prof0]  # (a library built before a slot existed reports fewer)
    dominant = max(kernel_slots, key=lambda s: prof0[s][0])
    stage_slots = [s for s in codec.SLOTS if s.startswith("stage.")]
    timed_slots = enc_slots if args.profile_all else (dominant, *stage_slots)
    codec.prof_enable(codec.slot_mask(*timed_slots))

    for _ in range(args.warmup):
        step()
    flush()
    torch.cuda.synchronize()
    codec.prof_reset()

    # ---- timed region ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    flush()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = codec.prof_read()

    value = global_total * args.steps / elapsed / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    dms, dcnt, dbytes = prof[dominant]
    avg_ms = dms / max(1, dcnt)
    bytes_per_launch = dbytes / max(1, dcnt)
    achieved = bytes_per_launch / (avg_ms / 1e3) / 1e9 if avg_ms > 0 else 0.0

    line = None
    if rank == 0:
        H, O, P = result["stream"]
        result["crc"] = int(result["crc_t"].item()) & 0xFFFFFFFF
        off_h = O.cpu().numpy()
        hdr_h = H.cpu().numpy()
        payload_bytes = int(off_h[nbg])
        rle_bytes = int(hdr_h[:, 260:264].copy().view(np.uint32).sum())
        pipeline_alg = 14 * global_total + 3 * rle_bytes + payload_bytes + 267 * nbg  # SURVEY 8.1 row d
        stage_ms = {s.split(".")[1]: round(prof[s][0] / args.steps, 3) for s in stage_slots}  # device ms per step (a stage may open several scopes per step)
        check, secondary = None, {}
        if not args.no_check:
            # decode the assembled global stream; its chunk-stream CRC must equal the merged shares
            # (every rank's input took part), and the blocks this rank holds must come back exactly
            out = codec.decode(H, O, P, global_total, bs)
            torch.cuda.synchronize()
            crc_dec = codec.chunks_crc32c(out, H, bs)
            mine_ok = all(torch.equal(out[g * bs:g * bs + min(bs, global_total - g * bs)], d[i * bs:i * bs + min(bs, my_bytes - i * bs)])
                          for i, g in enumerate(my_blocks))
            check = bool(crc_dec == result["crc"] and mine_ok)
            secondary["crc32c_chunk_stream"] = f"{result['crc']:08x}"
            if not args.no_secondary and world == 1:
                t1 = time.perf_counter()
                for _ in range(3):
                    codec.decode(H, O, P, global_total, bs, out=out)
                torch.cuda.synchronize()
                secondary["decode_GBps"] = round(3 * global_total / (time.perf_counter() - t1) / 1e9, 4)
                # decode roofline: stage times and the largest decode kernel, from one more decode
                # with every decode slot timed (HIP events on the decode's stream)
                dec_slots = [s for s in codec.SLOTS if s.startswith("dec.")]
                codec.prof_enable(codec.slot_mask(*dec_slots))
                codec.prof_reset()
                codec.decode(H, O, P, global_total, bs, out=out)
                torch.cuda.synchronize()
                dp = codec.prof_read()
                codec.prof_enable(0)
                dk = max(codec.DECODE_KERNELS, key=lambda s: dp[s][0])
                dms = dp[dk][0] / max(1, dp[dk][1])
                dach = dp[dk][2] / max(1, dp[dk][1]) / (dms / 1e3) / 1e9 if dms > 0 else 0.0
                secondary["decode_stage_ms"] = {s.split(".")[1]: round(dp[s][0], 3) for s in ("dec.huffman", "dec.rle", "dec.mtf", "dec.ibwt")}
                secondary["decode_roofline"] = {
                    "bound": "hbm", "kernel": dk, "achieved": round(dach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(dach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(dms, 4),
                    "algorithmic_bytes_per_launch": int(dp[dk][2] / max(1, dp[dk][1])),
                    "kernels_ms": {s: round(dp[s][0] / max(1, dp[s][1]), 4) for s in codec.DECODE_KERNELS}}
            del out
        if not args.no_secondary and world == 1 and len(batches) == 1:
            codec2 = bra.BlockCodec(local)
            secondary.update(pcie_inclusive(codec, data_np, d, bs, nb, hdr, off, pay, payload_bytes, work_stream, args.pcie_batches, codec2))
            codec2.close()
            secondary.update(pcie_stream(bra, codec, data_np, args.kind, bs, args.pcie_stream))

        line = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": f"{nbg} x {bs} B {args.kind} blocks ({global_total >> 20} MiB global, "
                            f"{'fixed total' if strong else f'{args.bytes_per_gpu >> 20} MiB per GPU'}; {WORKLOADS[args.kind]}), "
                            "encode BWT+MTF+RLE+Huffman + chunk-stream CRC32C + chunks assembled in block order on rank 0, "
                            "inputs resident in HBM",
                "block_size": bs,
                "global_bytes": global_total,
                "batches_per_rank": len(batches),
                "parallelism": f"dp{world}: block b on GPU b mod {world} (round robin)"
                               + ((f", RCCL gather of compressed chunks + CRC shares to rank 0 ({args.gather_mode} sizes)" if args.backend == "nccl" else
                                  f", {args.backend} gather through host copies (ranks sharing a GPU: rehearsal, not a scaling number)")
                                 if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dominant,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "avg_launch_ms": round(avg_ms, 4),
                "launches": dcnt,
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
            },
            "pipeline": {
                "stage_ms": stage_ms,
                "encode_device_ms": round(sum(stage_ms.values()), 3),
                "algorithmic_bytes": pipeline_alg,
                "hbm_frac": round(pipeline_alg / (ms_per_step / 1e3) / (HBM_PEAK_GBS * 1e9), 4),
                "ratio": round((payload_bytes + 267 * nbg) / global_total, 4),
                "rle_bytes": rle_bytes,
                "payload_bytes": payload_bytes,
                "roundtrip_bit_exact": check,
            },
            "secondary": secondary,
            "cpu_baseline": None,
        }
        if world > 1:
            # bytes that crossed to rank 0 per step (the last gather: headers, offsets, CRC shares,
            # payloads at their exact sizes or at the geometry's bound, --gather-mode)
            line["gather_bytes_per_step"] = int(gather.last_bytes)
            line["gather_mode"] = args.gather_mode
        if args.profile_all:
            line["kernels"] = {k: {"ms": round(v[0] / max(1, v[1]), 4), "launches": v[1], "GBps": round(v[2] / max(v[0], 1e-9) / 1e6, 1)}
                               for k, v in prof.items() if v[1]}
        if world == 1:
            cp = copy_peak_GBps(dev)
            line["roofline"]["measured_copy_peak"] = round(cp, 1)
            line["roofline"]["frac_of_copy_peak"] = round(line["roofline"]["achieved"] / cp, 4)
            line["pipeline"]["frac_of_copy_peak"] = round(pipeline_alg / (ms_per_step / 1e3) / (cp * 1e9), 4)
        # traffic: HBM bytes per launch of the same kernel slot on the same workload (input kind and
        # block size) from the committed rocprofv3 PMC passes (profiles/pmc_summary.json)
        pmc = os.path.join(ROOT, "profiles", "pmc_summary.json")
        if os.path.exists(pmc):
            try:
                wl = json.load(open(pmc)).get("workloads", {}).get(f"{args.kind}_{bs}", {})
                k = wl.get("kernels", {}).get(dominant)
                if k:
                    line["roofline"]["traffic"] = k.get("hbm_bytes_per_launch")
                    line["roofline"]["traffic_source"] = f"profiles/pmc_summary.json workloads.{args.kind}_{bs} ({wl.get('source', '?')})"
                # the compute side of the job kernels (sorting networks and string compares, not HBM
                # bound): the fraction of the chip's calibrated VALU issue ceiling the launch used
                # (valu_frac = SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs x 0.380 wave-instructions
                # per SIMD per cycle, the rate scripts/micro/valu_cal.hip reaches: profiles/
                # r06_valu_calibration.json) and VALU lane instructions per element the launch covers
                # (the job slots: their 11 algorithmic bytes per element; else the batch)
                valu = {}
                for slot in dict.fromkeys((dominant, "bwt.jobs", "bwt.mjobs")):
                    e = wl.get("kernels", {}).get(slot, {})
                    if "valu_frac" in e:
                        pe = prof0.get(slot)
                        elems = pe[2] / max(1, pe[1]) / 11.0 if slot.startswith("bwt.") and "jobs" in slot and pe and pe[2] else my_bytes
                        valu[slot] = {"valu_frac": e["valu_frac"],
                                      "valu_insts_per_element": round(e.get("valu_insts_per_launch", 0) * 64 / max(1.0, elems), 1)}
                if dominant in valu:
                    line["roofline"].update(valu[dominant])
                    if "jobs" in dominant and valu[dominant]["valu_frac"] > line["roofline"]["frac"]:
                        # the job kernels: VALU issue, not HBM, is the resource they use most of;
                        # achieved / peak / frac stay the HBM figures
                        line["roofline"]["bound"] = "valu"
                if valu:
                    line["roofline"]["valu"] = valu
            except (OSError, ValueError, AttributeError):
                pass
        if not args.no_check:
            line["reference_check"] = check_vs_reference(H, O, P, args.kind, bs, nbg, global_total, world, args.cpu_threads)
        if world == 1 and not args.no_cpu_baseline:
            gpu_chunks = []
            pay_h = P.cpu().numpy()
            for b in range(max(cpu_sample_sizes(nb, bs, args.cpu_threads))):
                pi, lens, osz, esz = bra.parse_header(hdr_h[b].tobytes())
                gpu_chunks.append((pi, lens, osz, esz, pay_h[off_h[b]:off_h[b] + esz].tobytes()))
            line["cpu_baseline"] = cpu_baseline(data_np, bs, args.cpu_threads, gpu_chunks)
        print(json.dumps(line), flush=True)
    codec.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
