"""Dynamic profile of the walk loop (k_walk / k_walk_seg / k_walk_refill, level 0 and bounce levels):
wave executions and active lanes of each part of a trip over one frame.  Needs the diagnostic build
(tools/build_variant.sh prof -DRT_WALK_PROF=1; RT_LIB=raytracer.js_amd/lib/librt_amd_prof.so).

    RT_LIB=... python tools/walk_profile.py [--config config3] [ENV=VAL ...]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer.js_amd", "python"))

import torch  # noqa: E402,F401

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

NAMES = ["trips", "walk_lanes", "head", "head_lanes", "emit", "emit_lanes", "stepin", "stepin_lanes", "exit",
         "exit_lanes", "move", "move_lanes", "walks", "waves"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("env", nargs="*")
    a = ap.parse_args()
    for kv in a.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
    factory, W, H, refmax = scenes.WORKLOADS[a.config]
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(refmax)
    ctx = rtamd.Context(0)
    ctx.upload(rtamd.build_scene(factory()))
    L = rtamd.load_library()
    fn = L.rt_debug_walk_profile
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 16)()
    buf_t = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    ctx.trace_rows_device(cam, cfg, 0, 1, H, buf_t.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert fn(buf, 1) == 0, "not a RT_WALK_PROF build"
    _, st = ctx.trace_rows_device(cam, cfg, 0, 1, H, buf_t.data_ptr(), s.cuda_stream, stats=True)   # counters only
    fn(buf, 1)
    ctx.trace_rows_device(cam, cfg, 0, 1, H, buf_t.data_ptr(), s.cuda_stream)
    s.synchronize()
    fn(buf, 0)
    v = dict(zip(NAMES, list(buf)[:14]))
    out = dict(config=a.config, env=a.env, raw=v, n_ret=st.n_ret, n_slot=st.n_slot)
    for part in ("head", "emit", "stepin", "exit", "move"):
        if v[part]:
            out[part + "_lanes_avg"] = round(v[part + "_lanes"] / v[part], 2)
            out[part + "_per_trip"] = round(v[part] / v["trips"], 3)
    out["trips_per_wave"] = round(v["trips"] / max(v["waves"], 1), 1)
    out["walking_lanes_avg"] = round(v["walk_lanes"] / max(v["trips"], 1), 2)
    out["lanes_at_start_avg"] = round(v["walks"] / max(v["waves"], 1), 2)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
