"""Device-side timeline of frames in flight (an RT_TL=1 build): F frames of one part
of n_parts on P contexts / streams, as tools/pipeline_probe.py runs them, then every launch's first
wave start and last wave end (100 MHz wall clock) from rt_debug_timeline.  Prints how many kernels
overlap, each kernel's mean time, and the gap between a launch and its stream predecessor's end.

    bash tools/build_variant.sh tl -DRT_TL=1
    RT_LIB=raytracer.js_amd/lib/librt_amd_tl.so python tools/tl_probe.py --parts 8 --inflight 16
"""
import os

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import argparse
import collections
import ctypes as C
import json
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer.js_amd", "python")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402


def read_timeline(lib, reset):
    n_max = 1 << 16
    se = (C.c_ulonglong * (4 * n_max))()
    names = C.create_string_buffer(64 * n_max)
    streams = (C.c_ulonglong * n_max)()
    lib.rt_debug_timeline.restype = C.c_int
    n = lib.rt_debug_timeline(n_max, se, names, streams, int(reset))
    if n < 0:
        raise RuntimeError("rt_debug_timeline: %d (an RT_TL=1 build is needed)" % n)
    out = []
    for i in range(n):
        nm = names.raw[64 * i:64 * i + 64].split(b"\0")[0].decode()
        out.append((se[4 * i], se[4 * i + 1], nm, streams[i], se[4 * i + 2], se[4 * i + 3]))
    return out


def analyse(recs, frames):
    recs = [r for r in recs if r[1] >= r[0] and r[0] != (1 << 64) - 1]   # launches whose waves ran
    if not recs:
        return {}
    t0 = min(r[0] for r in recs)
    t1 = max(r[1] for r in recs)
    ev = sorted([(r[0], 1) for r in recs] + [(r[1], -1) for r in recs])
    hist = collections.Counter()
    cur, prev = 0, ev[0][0]
    for t, d in ev:
        hist[cur] += t - prev
        cur += d
        prev = t
    tot = sum(hist.values()) or 1
    per = collections.defaultdict(list)
    wave_us = collections.defaultdict(float)
    waves = collections.defaultdict(int)
    for s, e, n, _, wt, wn in recs:
        per[n].append((e - s) * 1e-2)                                 # 10 ns ticks -> us
        wave_us[n] += wt * 1e-2
        waves[n] += wn
    gaps = collections.defaultdict(list)                              # launch start - previous launch end, same stream
    last = {}
    for s, e, n, st, *_ in sorted(recs):
        if st in last:
            gaps[n].append((s - last[st]) * 1e-2)
        last[st] = e
    return dict(
        wall_us_per_frame=round((t1 - t0) * 1e-2 / frames, 1),
        wave_ms_per_frame=round(sum(r[4] for r in recs) * 1e-5 / frames, 3),
        busy_frac=round(1 - hist.get(0, 0) / tot, 3),
        mean_concurrency=round(sum(k * v for k, v in hist.items()) / tot, 2),
        concurrency={k: round(v / tot, 3) for k, v in sorted(hist.items())},
        kernels={n: dict(calls=len(v), mean_us=round(float(np.mean(v)), 1), per_frame_us=round(sum(v) / frames, 1),
                         max_us=round(float(np.max(v)), 1),
                         waves_per_frame=round(waves[n] / frames, 1),
                         wave_ms_per_frame=round(wave_us[n] / frames / 1e3, 3),
                         gap_us=round(float(np.median(gaps[n])), 1) if gaps[n] else None)
                 for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--parts", type=int, nargs="*", default=[8])
    ap.add_argument("--inflight", type=int, nargs="*", default=[1, 16])
    ap.add_argument("--frames", type=int, default=48)
    ap.add_argument("--refmax", type=int, default=0)
    a = ap.parse_args()
    factory, W, H, refmax = scenes.WORKLOADS[a.config]
    refmax = a.refmax or refmax
    lib = rtamd.load_library()
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
        for p in a.inflight:
            for i in range(2 * p):
                ctxs[i % p].trace_rows_device(cam, cfg, 0, parts, 8, bufs[i % p].data_ptr(), streams[i % p].cuda_stream)
            torch.cuda.synchronize()
            read_timeline(lib, True)
            t0 = time.perf_counter()
            for i in range(a.frames):
                ctxs[i % p].trace_rows_device(cam, cfg, 0, parts, 8, bufs[i % p].data_ptr(), streams[i % p].cuda_stream)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.frames
            res = analyse(read_timeline(lib, True), a.frames)
            print(json.dumps(dict(parts=parts, inflight=p, host_ms_per_frame=round(dt * 1e3, 3), **res)), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
