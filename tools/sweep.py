"""Timing sweep of k_trace variants in one process (env knobs read at rt_create):
RT_OCC (occupancy variant), RT_DIAG (timing-only experiments), RT_NO_CULL, RT_BVH_SAH, RT_SPLIT, RT_CAND_CAP.

    python tools/sweep.py [--config config3] [--frames 5] VARIANT...   (VARIANT = "NAME:K=V,K=V")
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer.js_amd", "python"))

import torch  # noqa: E402,F401  (same HIP runtime as bench.py)

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

KNOBS = ("RT_OCC", "RT_DIAG", "RT_NO_CULL", "RT_BVH_SAH", "RT_SPLIT", "RT_CAND_CAP", "RT_CONT_GROUP", "RT_SPLIT_LEVELS",
         "RT_CLAIM_CHUNK", "RT_XCD", "RT_SHADE_OCC", "RT_SEG", "RT_SKIP", "RT_DERIVED", "RT_REFILL", "RT_LV_BLOCKS", "RT_SEG_MAX", "RT_REFILL_ALWAYS", "RT_TOP_LEVELS", "RT_BVH_LEAF", "RT_FUSE_MAX")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--refmax", type=int, default=None)
    ap.add_argument("variants", nargs="*", default=["base:"])
    a = ap.parse_args()
    factory, W, H, refmax = scenes.WORKLOADS[a.config]
    scene = rtamd.build_scene(factory())
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(a.refmax or refmax)
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    for v in a.variants:
        name, _, kv = v.partition(":")
        for k in KNOBS:
            os.environ.pop(k, None)
        for item in filter(None, kv.split(",")):
            k, _, val = item.partition("=")
            os.environ[k] = val
        ctx = rtamd.Context(0)
        ctx.upload(scene)
        _, st = ctx.trace_rows_device(cam, cfg, 0, 1, H, buf.data_ptr(), s.cuda_stream, stats=True)
        for _ in range(2):
            # each warm-up frame finishes before the next starts, so its work counters become the
            # grid hints / refill choices of the timed frames (the bench's steady state)
            ctx.trace_rows_device(cam, cfg, 0, 1, H, buf.data_ptr(), s.cuda_stream)
            s.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.frames):
            ctx.trace_rows_device(cam, cfg, 0, 1, H, buf.data_ptr(), s.cuda_stream)
        s.synchronize()
        wall = (time.perf_counter() - t0) / a.frames * 1e3
        kt = ctx.kernel_times(a.frames)
        extra = {"rgb_sum": int(buf.view(torch.int32).to(torch.int64).sum())}   # frame fingerprint
        if int(os.environ.get("RT_DIAG", "0")) & 8:
            tile = st.n_loc
            extra.update(lane_cycles_tile=tile, frac_walk=round(st.n_cull / tile, 3), frac_test=round(st.n_exact / tile, 3),
                         frac_other=round(1 - (st.n_cull + st.n_exact) / tile, 3))
        rec = dict(variant=name, env=kv, kernel_ms=round(float(kt.mean()), 3), kernel_min=round(float(kt.min()), 3),
                   wall_ms=round(wall, 3), mrays=round(st.segments / (wall * 1e-3) / 1e6, 2),
                   n_cull=st.n_cull, n_exact=st.n_exact, segments=st.segments, **extra)
        print(json.dumps(rec), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
