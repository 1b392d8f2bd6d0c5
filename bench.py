"""bench.py — Mrays/s and ms/frame of the MI355X render path (BASELINE.json metric).

A step is one frame: ray generation + trace + (N>1) RCCL gather of the row stripes to rank 0 and
de-interleave into the 1920x1080 frame.  The frame is split across ranks (strong scaling: the
frame size is fixed).  Inputs (scene, camera) are resident on the GPU before the timed region.

Frames in flight (--inflight P, default 16): each rank keeps P contexts, each on its own HIP
stream with its own frame buffers, and issues frame f on context f % P.  HIP maps streams onto
GPU_MAX_HW_QUEUES hardware queues (HIP's default is 4); the bench raises it to 16 before the HIP
runtime starts, so that 16 frames really run concurrently.  A frame's bounce level 1
is a latency-bound tail (few, long continuation rays) that the next frames' primary
passes fill.  Every one of the K timed frames is rendered and gathered completely inside the timed
region; `value` is their throughput.  A serial pass (one frame in flight) reports the per-frame
latency beside it (`serial`) and is what the roofline's kernel duration is measured on.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config config3]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0 (schema in the task contract) including `roofline` for the trace
kernel (algorithmic bytes per launch from the kernel's own work counters, SURVEY.md §8d, over the
HIP-event-timed kernel duration) and `cpu_baseline` (the oracle restatement, single-threaded, on a
bounded pixel sample of the same workload).
"""
import os

# hardware queues for the frames in flight, read once when the HIP runtime initialises: at least
# 16 (HIP's default, and the GPU box's setting, is 4)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import argparse
import csv
import glob
import json
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytracer.js_amd", "python"))

import rtamd  # noqa: E402  (after torch: share its HIP runtime)
from rtamd import scenes  # noqa: E402
from rtamd import abi  # noqa: E402
from rtamd.stripes import StripeGather  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# Algorithmic bytes per unit of work of the reference's algorithm (canonical f64
# layout) over the reference-equivalent counters: what the in-order entity scan would read.
BYTES_REF = dict(n_ret=48, n_slot=32, n_loc=40, n_sph=36, n_box=36, n_tri=76, n_hit=40, primary=12)
# Algorithmic bytes of the work k_trace actually performs: walker records as above,
# 32 B per cull-hierarchy box test, 80 B per exact entity test (record + rank), 44 B per hit (shade
# record + entity id), 36 B per pixel (24 B direction read + 12 B RGB store).
BYTES_KERNEL = dict(n_ret=48, n_slot=32, n_loc=40, n_cull=32, n_exact=80, n_hit=44, primary=36)


def algorithmic_bytes(counters, table):
    return sum(table[k] * counters[k] for k in table)


def cpu_baseline(spec, cam, cfg, budget_s):
    """Oracle restatement (plain C, 1 thread) on a random pixel sample; Mrays/s of traced segments."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    w, root = oracle.build_scene(spec)
    rng = np.random.default_rng(0)
    P = cam.width * cam.height
    order = rng.permutation(P).astype(np.int32)
    done, segs, t_used, chunk = 0, 0, 0.0, 2048
    while t_used < budget_s and done < P:
        pix = order[done:done + chunk]
        t0 = time.perf_counter()
        r = w.trace_frame(root, cam, cfg, pixels=pix, nthreads=1)
        t_used += time.perf_counter() - t0
        segs += r["counters"]["segments"]
        done += len(pix)
        chunk = min(chunk * 2, 65536) if t_used < budget_s / 4 else chunk
    # the same sample split over the host's CPU share (a worker split across all cores)
    nt = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    t0 = time.perf_counter()
    r = w.trace_frame(root, cam, cfg, pixels=order[:done], nthreads=nt)
    t_mt = time.perf_counter() - t0
    w.close()
    return dict(value=segs / t_used / 1e6, unit="Mrays/s", cores=1, kind="port",
                sample="%d random pixels of the %dx%d frame (%d segments) in %.1f s, oracle/rt_oracle.c, 1 thread"
                       % (done, cam.width, cam.height, segs, t_used),
                threaded=dict(value=r["counters"]["segments"] / t_mt / 1e6, unit="Mrays/s", cores=nt,
                              sample="the same pixels, %d threads, %.2f s" % (nt, t_mt)))


TRACE_KERNELS = ("k_walk", "k_first", "k_shade", "k_cont", "k_trace")
PMC_FRAMES = 4                 # frames the --pmc-child run traces (warmup 1 + steps 3)


def _pmc_pass(counter, config, stripe, timeout_s):
    """One rocprofv3 --pmc pass over a child bench run; counter total per frame over the trace
    kernels (the stats instantiation k_trace<true, ...> is not part of a frame)."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not on PATH"
    out = tempfile.mkdtemp(prefix="rt_pmc_")
    try:
        env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
        cmd = [prof, "--pmc", counter, "-d", out, "-o", "pmc", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--config", config,
               "--stripe", str(stripe), "--steps", "3", "--warmup", "1"]
        r = subprocess.run(cmd, env=env, timeout=timeout_s, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        if r.returncode != 0:
            tail = r.stdout.decode(errors="replace").strip().splitlines()[-3:]
            return None, "%s pass exit %d: %s" % (counter, r.returncode, " | ".join(tail))
        vals = []
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r["Kernel_Name"]
                    stats = "<true" in name or "ILb1E" in name
                    if any(k in name for k in TRACE_KERNELS) and not stats and r["Counter_Name"] == counter:
                        vals.append(float(r["Counter_Value"]))
        if not vals:
            return None, "%s pass: no trace-kernel rows in the counter CSV" % counter
        return sum(vals) / PMC_FRAMES, None
    except Exception as e:  # the bench line must not depend on the profiler
        return None, "%s pass: %r" % (counter, e)
    finally:
        shutil.rmtree(out, ignore_errors=True)


def hbm_traffic(config, stripe, timeout_s=300):
    """HBM bytes per frame's trace kernels from PMC (MI355X_MICROARCH.md HBM section): FETCH_SIZE
    and WRITE_SIZE in separate passes (TCC slots), both in KiB; FETCH_SIZE doubled (gfx950 tallies
    128-B requests at 64 B).  None when rocprofv3 or a pass is unavailable."""
    fetch, err = _pmc_pass("FETCH_SIZE", config, stripe, timeout_s)
    if err:
        return None, err
    write, err = _pmc_pass("WRITE_SIZE", config, stripe, timeout_s)
    if err:
        return None, err
    return dict(bytes=2 * fetch * 1024 + write * 1024, fetch_kib_raw=fetch, write_kib=write,
                method="rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes), summed over one frame's trace "
                       "kernels: 2*FETCH_SIZE + WRITE_SIZE"), None


def exposure_bench(ctx, frame, stream, reps=20):
    """The device-resident ExposureBuffer consumers on the frame just rendered:
    luminance statistics (two read passes, synchronising) and the RGBA8 tone map (one read, one
    write), as achieved HBM rate of their algorithmic bytes."""
    n = frame.shape[0] * frame.shape[1]
    sp = stream.cuda_stream
    st = ctx.exposure_stats_device(frame.data_ptr(), n, sp)
    t0 = time.perf_counter()
    for _ in range(reps):
        st = ctx.exposure_stats_device(frame.data_ptr(), n, sp)
    stats_ms = (time.perf_counter() - t0) / reps * 1e3
    lo, hi = rtamd.tonemap_range(abi.RT_TONEMAP_STDDEV, st)
    rgba = torch.empty(4 * n, dtype=torch.uint8, device=frame.device)
    ctx.tonemap_device(frame.data_ptr(), n, lo, hi, rgba.data_ptr(), sp)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        ctx.tonemap_device(frame.data_ptr(), n, lo, hi, rgba.data_ptr(), sp)
    e1.record(stream)
    e1.synchronize()
    tm_ms = e0.elapsed_time(e1) / reps
    stats_bytes, tm_bytes = 2 * 12 * n, 12 * n + 4 * n
    return dict(stats_ms=round(stats_ms, 4), stats_GBps=round(stats_bytes / (stats_ms * 1e-3) / 1e9, 1),
                stats_note="wall time incl. launch + 24-B readback + sync",
                tonemap_ms=round(tm_ms, 4), tonemap_GBps=round(tm_bytes / (tm_ms * 1e-3) / 1e9, 1),
                mean=st.mean, variance=st.variance, range=[lo, hi])


def pmc_child(args):
    """Minimal frame loop profiled by hbm_traffic(): no stats launch, no CPU baseline, no output."""
    factory, W, H, refmax = scenes.WORKLOADS[args.config]
    ctx = rtamd.Context(0)
    ctx.upload(rtamd.build_scene(factory()))
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(refmax)
    buf = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    for _ in range(PMC_FRAMES):
        ctx.trace_rows_device(cam, cfg, 0, 1, args.stripe, buf.data_ptr(), s.cuda_stream)
    s.synchronize()
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="config3", choices=sorted(scenes.WORKLOADS))
    ap.add_argument("--stripe", type=int, default=8, help="rows per stripe of the row-interleaved split")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle CPU work (0 = skip)")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes for roofline.traffic")
    ap.add_argument("--inflight", type=int, default=16, help="frames in flight per rank (contexts / streams)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.pmc_child:
        return pmc_child(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RT_BENCH_BACKEND") == "gloo":
        local %= torch.cuda.device_count()       # plumbing check: ranks may share the box's one GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("RT_BENCH_BACKEND", "nccl")   # "gloo": plumbing checks with ranks sharing a GPU
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))

    factory, W, H, refmax = scenes.WORKLOADS[args.config]
    spec = factory()
    t0 = time.perf_counter()
    scene = rtamd.build_scene(spec)
    build_s = time.perf_counter() - t0
    P = max(1, min(args.inflight, args.steps))
    ctxs = []
    for _ in range(P):
        c = rtamd.Context(local)
        c.upload(scene)
        ctxs.append(c)
    ctx = ctxs[0]
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(refmax)
    # explicit streams for librt launches, torch copies and the collectives (the legacy NULL
    # stream would not order against librt's non-blocking stream); frame f uses slot f % P
    streams = [torch.cuda.Stream(device=dev) for _ in range(P)]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    sgs = [StripeGather(H, W, rank, world, args.stripe, dev) for _ in range(P)]
    sg = sgs[0]
    local_buf = sg.local

    def step(f, inflight):
        i = f % inflight
        with torch.cuda.stream(streams[i]):
            ctxs[i].trace_rows_device(cam, cfg, rank, world, args.stripe, sgs[i].local.data_ptr(),
                                      streams[i].cuda_stream)
            sgs[i].gather()        # the collective waits for this stream; this stream for it

    def timed(inflight, steps, warmup):
        for f in range(warmup):
            step(f, inflight)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for f in range(steps):
            step(f, inflight)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # work counters of one frame (untimed STATS launch): segments and algorithmic bytes
    _, st = ctx.trace_rows_device(cam, cfg, rank, world, args.stripe, local_buf.data_ptr(), sp, stats=True)
    counters = dict(st.counters(), **st.work())
    names = st.COUNTERS + st.WORK
    ctr = torch.tensor([counters[k] for k in names], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(ctr)
    tot = dict(zip(names, ctr.tolist()))
    local_bytes = algorithmic_bytes(counters, BYTES_KERNEL)
    local_bytes_ref = algorithmic_bytes(counters, BYTES_REF)

    elapsed = timed(P, args.steps, max(args.warmup, P))
    # every in-flight slot rendered the same camera: their gathered frames must agree bit for bit
    same = all(torch.equal(sgs[i].frame.view(torch.int32), sgs[0].frame.view(torch.int32)) for i in range(1, P)) \
        if rank == 0 else None
    # N > 1: rank 0's gathered frame equals the whole frame rendered on its own GPU alone
    if world > 1 and rank == 0:
        whole = torch.zeros((H, W, 3), dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)
        ctx.trace_rows_device(cam, cfg, 0, 1, H, whole.data_ptr(), sp)
        torch.cuda.synchronize(dev)
        same = bool(same) and torch.equal(whole.view(torch.int32), sgs[0].frame.view(torch.int32))
    # serial pass: one frame in flight on context 0; its HIP events give the kernel duration
    elapsed_serial = timed(1, args.steps, 1) if P > 1 else elapsed
    kt = ctx.kernel_times(args.steps)
    k_ms = float(np.mean(kt)) if len(kt) else float("nan")

    ms_per_step = elapsed / args.steps * 1e3
    value = tot["segments"] * args.steps / elapsed / 1e6
    serial = dict(frames_in_flight=1, ms_per_frame=round(elapsed_serial / args.steps * 1e3, 4),
                  value=round(tot["segments"] * args.steps / elapsed_serial / 1e6, 3), unit="Mrays/s")
    achieved = local_bytes / (k_ms * 1e-3) / 1e9 if k_ms == k_ms and k_ms > 0 else None
    roofline = dict(bound="hbm", achieved=achieved, peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=(achieved / HBM_PEAK_GBS) if achieved else None, traffic=None,
                    kernel="trace (k_walk + k_first + k_shade per bounce level, k_cont)", kernel_ms=k_ms,
                    bytes_per_launch=local_bytes,
                    bytes_formula="48*n_ret+32*n_slot+40*n_loc+32*n_cull+80*n_exact+44*n_hit+36*primary",
                    bytes_reference_equivalent=local_bytes_ref,
                    reference_equivalent_formula="SURVEY 8d: 48*n_ret+32*n_slot+40*n_loc+36*n_sph+36*n_box+76*n_tri+40*n_hit+12*primary")

    # PCIe-inclusive rate of the host-buffer entry point (rt_trace_frame: RGB copied back to a host
    # Float32Array-sized buffer each frame) — reported beside `value`, never as it
    host = None
    if rank == 0 and world == 1:
        rgb_host = np.zeros(W * H * 3, np.float32)
        ctx.trace_frame(cam, cfg, rgb=rgb_host, ids=False, stats=False)
        t0 = time.perf_counter()
        n_host = 3
        for _ in range(n_host):
            ctx.trace_frame(cam, cfg, rgb=rgb_host, ids=False, stats=False)
        host_ms = (time.perf_counter() - t0) / n_host * 1e3
        host = dict(entry="rt_trace_frame (host RGB buffer)", ms_per_frame=round(host_ms, 3),
                    value=round(tot["segments"] / (host_ms * 1e-3) / 1e6, 3), unit="Mrays/s")

    exposure = exposure_bench(ctx, sg.frame, stream) if rank == 0 else None

    traffic = None
    if rank == 0 and world == 1 and not args.no_traffic:
        traffic, err = hbm_traffic(args.config, args.stripe)
        if traffic is not None:
            roofline["traffic"] = traffic["bytes"]
            roofline["traffic_detail"] = traffic
        else:
            roofline["traffic_note"] = err

    cpu = None
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        cpu = cpu_baseline(spec, cam, cfg, args.cpu_budget)

    if rank == 0:
        rec = {
            "metric": "Mrays/s (whole node) at %dx%d" % (W, H),
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 seed 42 scene, BASELINE.json %s)" % args.config,
            "config": {"workload": args.config, "scene": spec.name, "width": W, "height": H, "refmax": refmax,
                       "entities": int(len(spec.entities)), "octree_nodes": int(scene.n_nodes),
                       "segments_per_frame": tot["segments"], "parallelism": "rows%d/stripe%d" % (world, args.stripe),
                       "frames_in_flight": P, "frames_identical": same,
                       "counters": tot, "scene_build_s": round(build_s, 3)},
            "roofline": roofline,
            "serial": serial,
            "cpu_baseline": cpu,
            "pcie_inclusive": host,
            "exposure": exposure,
            "mpixels_per_s": round(W * H * args.steps / elapsed / 1e6, 3),
        }
        print(json.dumps(rec), flush=True)
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
