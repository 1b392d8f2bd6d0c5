"""PCIe copy rates of a 1080p ExposureBuffer (1920*1080*3 f32 = 24.9 MB) between the device and
pageable / pinned host memory, as rt_trace_frame's host copies see them.

    python tools/copy_probe.py
"""
import json
import time

import numpy as np
import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    n = 1920 * 1080 * 3
    dev = torch.zeros(n, dtype=torch.float32, device="cuda")
    page = torch.from_numpy(np.ones(n, np.float32))
    pin = torch.ones(n, dtype=torch.float32).pin_memory()
    nb = n * 4
    for name, fn in [("h2d_pageable", lambda: dev.copy_(page, non_blocking=True)),
                     ("h2d_pinned", lambda: dev.copy_(pin, non_blocking=True)),
                     ("d2h_pageable", lambda: page.copy_(dev, non_blocking=True)),
                     ("d2h_pinned", lambda: pin.copy_(dev, non_blocking=True)),
                     ("host_memcpy", lambda: page.numpy().__setitem__(slice(None), pin.numpy()))]:
        s = timed(fn)
        print(json.dumps(dict(copy=name, ms=round(s * 1e3, 3), GBps=round(nb / s / 1e9, 1))), flush=True)


if __name__ == "__main__":
    main()
