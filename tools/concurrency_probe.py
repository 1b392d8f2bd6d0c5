"""How many kernels from different streams run at once: K streams each launch one long, tiny
(1-block) spin kernel; the wall time is ~ceil(K / C) spins when at most C kernels run concurrently.
Also a "busy" variant where each kernel has B blocks.  For DESIGN.md §7 (frames in flight).

    python tools/concurrency_probe.py [--cycles 2000000]
"""
import os

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=2_000_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(device=dev) for _ in range(32)]
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(a.cycles)
    torch.cuda.synchronize()
    one = time.perf_counter() - t0
    for k in (1, 2, 3, 4, 5, 6, 8, 12, 16, 24, 32):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            with torch.cuda.stream(streams[i]):
                torch.cuda._sleep(a.cycles)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps(dict(streams=k, wall_ms=round(dt * 1e3, 3), spins=round(dt / one, 2),
                              hw_queues=os.environ.get("GPU_MAX_HW_QUEUES"))), flush=True)


if __name__ == "__main__":
    main()
