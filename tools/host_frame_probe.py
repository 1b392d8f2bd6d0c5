"""rt_trace_frame into a host buffer (the JS drop-in's call) as row bands: median ms per frame for
several RT_BANDS values, into pageable and into pinned host memory.

python tools/host_frame_probe.py [--config config3] [--bands 1 2 4] [--frames 10]
"""
import os

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import argparse
import json
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer.js_amd", "python")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--bands", type=int, nargs="*", default=[1, 2, 4])
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--pinned", action="store_true", help="also time a pinned destination buffer")
    ap.add_argument("--orders", type=int, nargs="*", default=[3], help="RT_BAND_ORDER values")
    a = ap.parse_args()
    factory, W, H, refmax = scenes.WORKLOADS[a.config]
    scene = rtamd.build_scene(factory())
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(refmax)
    torch.cuda.init()
    dests = [("pageable", np.zeros(W * H * 3, np.float32))]
    if a.pinned:
        dests.append(("pinned", torch.zeros(W * H * 3, dtype=torch.float32, pin_memory=True).numpy()))
    ref = None
    for nb, order in [(nb, o) for nb in a.bands for o in (a.orders if nb > 1 else [0])]:
        os.environ["RT_BANDS"] = str(nb)
        os.environ["RT_BAND_ORDER"] = str(order)
        c = rtamd.Context(0)
        c.upload(scene)
        for name, rgb in dests:
            for _ in range(3):
                c.trace_frame(cam, cfg, rgb=rgb, ids=False, stats=False)
            ts = []
            for _ in range(a.frames):
                t0 = time.perf_counter()
                c.trace_frame(cam, cfg, rgb=rgb, ids=False, stats=False)
                ts.append((time.perf_counter() - t0) * 1e3)
            if ref is None:
                ref = rgb.copy()
            print(json.dumps(dict(bands=nb, order=order, dest=name, ms_median=round(float(np.median(ts)), 3),
                                  ms_min=round(min(ts), 3), identical=bool(np.array_equal(ref, rgb)))), flush=True)
        c.close()


if __name__ == "__main__":
    main()
