"""k_frame_start alone (rt_debug_camera_dirs: the launch with the trace skipped, then a D2H of the
directions), N times on the library in RT_LIB, for same-box A/B under rocprofv3 --kernel-trace --stats.

    RT_LIB=raytracer.js_amd/lib/librt_amd_fsptr.so rocprofv3 --kernel-trace --stats -d out -- \\
        python3 tools/frame_start_ab.py --frames 40
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer.js_amd", "python")]

import numpy as np  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--frames", type=int, default=40)
    a = ap.parse_args()
    factory, W, H, _ = scenes.WORKLOADS[a.config]
    ctx = rtamd.Context(0)
    ctx.upload(rtamd.build_scene(factory()))
    cam = scenes.make_camera(W, H)
    dirs = np.zeros(3 * W * H, np.float64)
    for _ in range(a.frames):
        rc = ctx.L.rt_debug_camera_dirs(ctx.h, C.byref(cam), dirs.ctypes.data_as(C.POINTER(C.c_double)))
        assert rc == 0, rc
    print("frames", a.frames, "lib", os.environ.get("RT_LIB", "default"), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
