"""The N > 1 bench path on one GPU (ranks sharing the device, gloo exchange through host copies).

The scaling run itself (RCCL over xGMI, one rank per GPU) belongs to the driver's 8-GPU node; this
rehearses everything else of `bench.py --gpus N` on the real device: torchrun spawning, round-robin
sharding (block b on rank b mod N), per-rank encodes, the chunk gather to rank 0, the on-device
assembly in global block order and the merged CRC shares -- and checks every global block's record
against the reference digests (tests/golden/digests.json) and a live reference encode of sampled
blocks from every rank.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_bench_sharded_path_on_one_gpu(world):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--backend", "gloo", "--steps", "1", "--warmup", "0",
           "--no-cpu-baseline", "--no-secondary", "--bytes-per-gpu", str(64 << 20)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world
    check = line["reference_check"]
    assert check["live"]["bit_exact"], check["live"]
    assert len(check["live"]["ranks"]) >= 2
    if "digests" in check:  # the digests cover the default text workload's global blocks
        assert check["digests"]["bit_exact"], check["digests"]
    assert line["pipeline"]["roundtrip_bit_exact"]
