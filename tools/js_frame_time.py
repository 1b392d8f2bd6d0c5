"""The JS drop-in's trace_frame() wall time (node -> N-API -> librt_amd.so, ExposureBuffer.pixels
filled): a BASELINE config's scene dumped to JSON, built as reference-shaped objects by
tests/js/run_dropin.js, then N frames timed without and with options.stats (work counters).

python tools/js_frame_time.py [--config config3] [--frames 10]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer.js_amd", "python")]

import numpy as np  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

RUNNER = os.path.join(ROOT, "tests", "js", "run_dropin.js")


def _dump(tmp_path, spec, cam, cfg):
    """The scene, camera and config as the JSON run_dropin.js inflates into reference-shaped objects
    (the same format as tests/test_js_dropin.py writes)."""
    s = rtamd.build_scene(spec)
    sc = {k: getattr(s, k).tolist() for k in ("node_pos", "node_size", "node_parent", "node_child", "node_ent_begin",
                                             "node_ent_count", "list_entity", "ent_type", "ent_geom", "ent_shade",
                                             "ent_substance", "substance_ri")}
    sc["shades"] = [dict(response=int(x["response"]), light=int(x["light"]), mirror=int(x["mirror"]),
                         roughness=float(x["roughness"]), image=int(x["image"]), rgb=[float(v) for v in x["rgb"]])
                    for x in s.shades]
    sc["images"] = [dict(width=int(im.shape[1]), height=int(im.shape[0]), rgb=im.reshape(-1).tolist()) for im in s.images]
    sc["cam"] = dict(width=cam.width, height=cam.height, pos=list(cam.pos), fr=list(cam.fr), lf=list(cam.lf),
                     up=list(cam.up), scan_h=list(cam.scan_h), scan_v=list(cam.scan_v))
    sc["cfg"] = dict(refmax=cfg.refmax, default_substance=cfg.default_substance, atten=cfg.distance_attenuation_factor,
                     sky=list(cfg.sky_rgb), sky_image=int(cfg.sky_image))
    p = tmp_path / "scene.json"
    p.write_text(json.dumps(sc))
    return str(p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--frames", type=int, default=10)
    a = ap.parse_args()
    factory, W, H, refmax = scenes.WORKLOADS[a.config]
    with tempfile.TemporaryDirectory() as td:
        path = _dump(Path(td), factory(), scenes.make_camera(W, H), scenes.make_config(refmax))
        r = subprocess.run(["node", "--max-old-space-size=16384", RUNNER, path, os.path.join(td, "out"),
                            "--repeat", str(a.frames)], capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            sys.exit(r.stdout[-2000:] + r.stderr[-2000:])
        rep = json.loads(Path(td, "out.repeat.json").read_text())
    med = {k: float(np.median(v)) for k, v in rep.items()}
    print(json.dumps(dict(config=a.config, frames=a.frames, js_trace_frame_ms_median=round(med["frame_ms"], 3),
                          js_trace_frame_ms_median_with_stats=round(med["frame_ms_stats"], 3), raw=rep)))


if __name__ == "__main__":
    main()
