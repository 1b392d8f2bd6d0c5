"""Driver of oracle/js/rt_path.js, the render path restated in JavaScript on Node (V8).

TEST INFRASTRUCTURE / CPU BASELINE ONLY: tests/test_js_baseline.py checks it against the C oracle,
and bench.py's cpu_baseline leg times it (BASELINE.md "CPU-baseline plan": the path in JS on the
host cores, one thread and a worker_threads split).  The product path never imports this module.

export(scene, cam, cfg, pixels, dir) writes the linearised scene (rtamd SceneArrays: DFS nodes with
their EntitySet-ordered lists, entity geometry, shades), the camera, the config and the pixel sample;
run(dir, threads) runs node on it and returns the per-pixel results and the timing line.
"""
import json
import os
import shutil
import signal
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = os.path.join(HERE, "js", "rt_path.js")


def node_binary():
    """Path of the node executable, or None."""
    return shutil.which("node")


def _vec(v, n):
    return [float(v[i]) for i in range(n)]


def export(scene, cam, cfg, pixels, out_dir, lights=(), ambient=0.0):
    """lights / ambient: shadow rays, a build extension (include/rt.h rt_set_lights)."""
    os.makedirs(out_dir, exist_ok=True)
    arrays = dict(node_pos=(scene.node_pos, "<f8"), node_size=(scene.node_size, "<f8"),
                  node_parent=(scene.node_parent, "<i4"), node_child=(scene.node_child, "<i4"),
                  node_ent_begin=(scene.node_ent_begin, "<i4"), node_ent_count=(scene.node_ent_count, "<i4"),
                  list_entity=(scene.list_entity, "<i4"), ent_type=(scene.ent_type, "<i4"),
                  ent_geom=(scene.ent_geom, "<f8"), ent_shade=(scene.ent_shade, "<i4"),
                  ent_substance=(scene.ent_substance, "<i4"), pixels=(np.asarray(pixels), "<i4"))
    for name, (a, dt) in arrays.items():
        np.ascontiguousarray(a, dtype=dt).tofile(os.path.join(out_dir, name + ".bin"))
    shades = [dict(response=int(s["response"]), light=int(s["light"]), mirror=int(s["mirror"]),
                   image=int(s["image"]), roughness=float(s["roughness"]), rgb=[float(x) for x in s["rgb"]])
              for s in scene.shades]
    man = dict(
        camera=dict(width=int(cam.width), height=int(cam.height), pos=_vec(cam.pos, 3), fr=_vec(cam.fr, 3),
                    lf=_vec(cam.lf, 3), up=_vec(cam.up, 3), scan_h=_vec(cam.scan_h, 2), scan_v=_vec(cam.scan_v, 2)),
        config=dict(refmax=int(cfg.refmax), default_substance=int(cfg.default_substance),
                    sky_rgb=_vec(cfg.sky_rgb, 3), distance_attenuation_factor=float(cfg.distance_attenuation_factor),
                    col_weight=float(cfg.col_weight), sky_image=int(cfg.sky_image)),
        shades=shades, substance_ri=[float(x) for x in scene.substance_ri],
        lights=[dict(pos=[float(x) for x in p], rgb=[float(x) for x in c]) for p, c in lights],
        ambient=float(ambient))
    with open(os.path.join(out_dir, "manifest.json"), "w") as f:
        json.dump(man, f)                       # floats as repr: they parse back to the same doubles


def run(out_dir, threads=1, repeat=1, timeout=600):
    """Run node on an exported directory; returns (timing dict, results dict of per-sample arrays)."""
    node = node_binary()
    if node is None:
        raise RuntimeError("node not found")
    # own session, output in files: at the timeout the whole group is killed and nothing can hold a
    # pipe open (bench.py bounds its total wall time with these limits)
    with tempfile.TemporaryFile() as fo, tempfile.TemporaryFile() as fe:
        p = subprocess.Popen([node, "--max-old-space-size=8192", SCRIPT, out_dir, "--threads", str(threads),
                              "--repeat", str(repeat)], stdout=fo, stderr=fe, start_new_session=True)
        try:
            rc = p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
            raise
        fo.seek(0)
        fe.seek(0)
        stdout, stderr = fo.read().decode(errors="replace"), fe.read().decode(errors="replace")
    if rc != 0:
        raise RuntimeError("rt_path.js failed (%d): %s" % (rc, stderr[-2000:]))
    info = json.loads(stdout.strip().splitlines()[-1])
    rd = lambda n, dt: np.fromfile(os.path.join(out_dir, "out_%s.bin" % n), dtype=dt)
    res = dict(rgb=rd("rgb", "<f4").reshape(-1, 3), hit_entity=rd("hit_entity", "<i4"),
               hit_node=rd("hit_node", "<i4"), segments=rd("segments", "<i4"), status=rd("status", "u1"))
    return info, res
