"""Config 5 device frames with and without two lights (tools/gpu_r5v49.sh runs it under rocprofv3
--kernel-trace): which passes a lit frame lengthens, level by level."""
import sys
sys.path.insert(0, "raytracer.js_amd/python")
sys.path.insert(0, ".")
import torch, rtamd
from rtamd import scenes
import bench

factory, W, H, refmax = scenes.WORKLOADS["config5"]
scene = rtamd.build_scene(factory())
cam, cfg = scenes.make_camera(W, H), scenes.make_config(refmax)
buf = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.Stream()
for lit in (False, True):
    ctx = rtamd.Context(0)
    ctx.upload(scene)
    if lit:
        ctx.set_lights(bench.BENCH_LIGHTS[:2], 0.1)
    for i in range(3):
        ctx.trace_rows_device(cam, cfg, 0, 1, H, buf.data_ptr(), s.cuda_stream)
        s.synchronize()
    print("lit" if lit else "unlit", "done", flush=True)
    ctx.close()
