"""The transfer-inclusive encode of bench.py alone (SURVEY 8.1(d) secondary), for a rocprofv3
kernel + memory-copy trace that shows the copies under the kernels (measurement only):

    rocprofv3 --kernel-trace --memory-copy-trace -d <dir> -o run --output-format csv -- \
        python3 scripts/pcie_trace.py [batches | b1,b2,... | stream[:S]] [kind] [block_size]

Prints the JSON of bench.pcie_inclusive (serial and overlapped GB/s)."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench

    # batches: a count (equal batches), a comma-separated list of batch sizes in blocks, or
    # "stream[:S]" (S batches of 256 MiB through the pipelined API, bench.pcie_stream)
    arg = sys.argv[1] if len(sys.argv) > 1 else "2"
    if arg.startswith("stream"):
        kind = sys.argv[2] if len(sys.argv) > 2 else "text"
        bs = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
        bra = importlib.import_module("br-archive_amd")
        data_np = bra.synth_fill(bench.KINDS[kind], 256 << 20, bs)
        codec = bra.BlockCodec(0)
        res = bench.pcie_stream(bra, codec, data_np, kind, bs, int(arg.split(":")[1]) if ":" in arg else 4)
        codec.close()
        print(json.dumps(res), flush=True)
        return
    split = [int(v) for v in arg.split(",")] if "," in arg else None
    nbatch = len(split) if split else int(arg)
    import torch

    kind = sys.argv[2] if len(sys.argv) > 2 else "text"
    bs = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
    bra = importlib.import_module("br-archive_amd")
    total = 256 << 20
    nb = total // bs
    data_np = bra.synth_fill(bench.KINDS[kind], total, bs)
    d = torch.from_numpy(data_np).cuda()
    codec = bra.BlockCodec(0)
    hdr = torch.empty((nb, bra.HEADER_BYTES), dtype=torch.uint8, device=d.device)
    off = torch.empty((nb + 1,), dtype=torch.int64, device=d.device)
    pay = torch.empty((int(total * 1.25) + 64 * nb + 65536,), dtype=torch.uint8, device=d.device)
    ws = torch.cuda.Stream()
    with torch.cuda.stream(ws):
        codec.encode(d, bs, hdr, off, pay, stream=ws)  # warm-up (allocations, geometry upload)
    torch.cuda.synchronize()
    payload_bytes = int(off[nb].item())
    codec2 = bra.BlockCodec(0)
    res = bench.pcie_inclusive(codec, data_np, d, bs, nb, hdr, off, pay, payload_bytes, ws, nbatch, codec2, split)
    codec2.close()
    res["device_resident_reference"] = "bench.py value (same input, one 256 MiB batch)"
    print(json.dumps(res), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
