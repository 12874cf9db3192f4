"""Cross-stream event wait after a host-to-device copy (measurement only).
Two 128 MiB pinned copies are queued on one copy stream with an event after each; a kernel on a
work stream waits on event 0.  We note when the host sees event 0, event 1 and the kernel complete.
Cases: the copy stream and the work stream among `extra` other streams of the process (HIP maps
streams onto at most GPU_MAX_HW_QUEUES hardware queues per priority, round robin), and the copy
stream created with high priority (its own queue pool)."""
import json
import time

import torch

n = 128 << 20
h = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(2)]
d = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(2)]
x = torch.zeros(1, device="cuda")


def case(name, cs, ws):
    for _ in range(2):
        torch.cuda.synchronize()
        ev = [torch.cuda.Event() for _ in range(2)]
        t0 = time.perf_counter()
        with torch.cuda.stream(cs):
            for k in range(2):
                d[k].copy_(h[k], non_blocking=True)
                ev[k].record(cs)
        ws.wait_event(ev[0])
        with torch.cuda.stream(ws):
            x.add_(1)
            kd = torch.cuda.Event()
            kd.record(ws)
        seen = {}
        while len(seen) < 3:
            now = time.perf_counter() - t0
            for nm, e in (("ev0", ev[0]), ("ev1", ev[1]), ("kernel_after_ev0", kd)):
                if nm not in seen and e.query():
                    seen[nm] = round(now * 1e3, 3)
    print(json.dumps({"case": name, "host_ms": seen}), flush=True)


pool = [torch.cuda.Stream() for _ in range(8)]
for k in range(8):  # touch every stream so each has its hardware queue
    with torch.cuda.stream(pool[k]):
        x.add_(0)
torch.cuda.synchronize()
for j in range(1, 8):
    case(f"copy on pool[0], work on pool[{j}]", pool[0], pool[j])
hp = torch.cuda.Stream(priority=-1)
case("copy on high-priority stream, work on pool[4]", hp, pool[4])
case("copy on high-priority stream, work on pool[0]", hp, pool[0])
