"""Latency of small synchronous frames (the reference's 128^2 demo canvas, BASELINE config 1 at 256^2):
rt_trace_frame into a host buffer, median wall ms over --frames, per variant of env knobs read at
rt_create (e.g. RT_SPLIT=0 for the fused one-kernel trace).  Prints one JSON line per (size, variant)
with the frame's fingerprint, so variants can be checked for identical pixels.

python tools/small_frame_probe.py [--sizes 128 256] [--frames 50] VARIANT...   (VARIANT = "NAME:K=V,K=V")
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer.js_amd", "python")]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

KNOBS = ("RT_SPLIT", "RT_HINTS", "RT_BANDS", "RT_BAND_MIN", "RT_SEG", "RT_LV_BLOCKS", "RT_OCC", "RT_CONT_GROUP",
         "RT_FUSE_MAX", "RT_FUSE_LIST")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="*", default=[128, 256])
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--refmax", type=int, default=2)
    ap.add_argument("--scene", default="config1", help="config1 (8 spheres), config2 (10k triangles), config3 "
                    "(100k triangles + 1k spheres) or smallN (scenes.small_random(N): 250 mixed entities)")
    ap.add_argument("variants", nargs="*", default=["base:"])
    a = ap.parse_args()
    if a.scene.startswith("small"):
        spec = scenes.small_random(int(a.scene[5:] or 4))
    else:
        spec = {"config1": scenes.config1_spheres, "config2": scenes.config2, "config3": scenes.config3}[a.scene]()
    scene = rtamd.build_scene(spec)
    cfg = scenes.make_config(a.refmax)
    for n in a.sizes:
        cam = scenes.make_camera(n, n)
        for v in a.variants:
            name, _, kv = v.partition(":")
            for k in KNOBS:
                os.environ.pop(k, None)
            for item in filter(None, kv.split(",")):
                k, _, val = item.partition("=")
                os.environ[k] = val
            c = rtamd.Context(0)
            c.upload(scene)
            rgb = np.zeros(n * n * 3, np.float32)
            for _ in range(5):
                c.trace_frame(cam, cfg, rgb=rgb, ids=False, stats=False)
            ts = []
            for _ in range(a.frames):
                t0 = time.perf_counter()
                c.trace_frame(cam, cfg, rgb=rgb, ids=False, stats=False)
                ts.append((time.perf_counter() - t0) * 1e3)
            print(json.dumps(dict(size=n, variant=name, env=kv, ms_median=round(float(np.median(ts)), 4),
                                  ms_min=round(min(ts), 4), ms_p90=round(float(np.percentile(ts, 90)), 4),
                                  rgb_sum=int(rgb.view(np.int32).astype(np.int64).sum()))), flush=True)
            c.close()


if __name__ == "__main__":
    main()
