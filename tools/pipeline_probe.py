"""Frames in flight: throughput of rt_trace_rows_device with P contexts on P streams, alternating
frames, for a part of n_parts row stripes (n_parts = 8 models one GPU of an 8-GPU node).

python tools/pipeline_probe.py [--parts 1 8] [--inflight 1 2 3] [--frames 30]
"""
import os

# hardware queues for the frames in flight, read once when the HIP runtime initialises: at least
# 16 (HIP's default, and the GPU box's setting, is 4)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import argparse
import json
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer.js_amd", "python")]

import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--parts", type=int, nargs="*", default=[1, 8])
    ap.add_argument("--inflight", type=int, nargs="*", default=[1, 2, 3])
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--refmax", type=int, default=0, help="override the workload's refmax (0: keep)")
    a = ap.parse_args()
    factory, W, H, refmax = scenes.WORKLOADS[a.config]
    refmax = a.refmax or refmax
    scene = rtamd.build_scene(factory())
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(refmax)
    dev = torch.device("cuda", 0)
    ctxs = []
    for _ in range(max(a.inflight)):
        c = rtamd.Context(0)
        c.upload(scene)
        ctxs.append(c)
    streams = [torch.cuda.Stream(device=dev) for _ in ctxs]
    bufs = [torch.zeros((H, W, 3), dtype=torch.float32, device=dev) for _ in ctxs]
    torch.cuda.synchronize()
    for parts in a.parts:
        _, st = ctxs[0].trace_rows_device(cam, cfg, 0, parts, 8, bufs[0].data_ptr(), streams[0].cuda_stream, stats=True)
        seg = st.segments
        for p in a.inflight:
            for i in range(2 * p):
                ctxs[i % p].trace_rows_device(cam, cfg, 0, parts, 8, bufs[i % p].data_ptr(), streams[i % p].cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.frames):
                ctxs[i % p].trace_rows_device(cam, cfg, 0, parts, 8, bufs[i % p].data_ptr(), streams[i % p].cuda_stream)
            t_sub = time.perf_counter() - t0                 # host time to submit (launches return early)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.frames
            print(json.dumps(dict(parts=parts, inflight=p, ms_per_frame=round(dt * 1e3, 3),
                                  mrays_per_gpu=round(seg / dt / 1e6, 1),
                                  host_submit_ms_per_frame=round(t_sub / a.frames * 1e3, 3))), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
