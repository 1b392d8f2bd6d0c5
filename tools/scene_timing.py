"""Scene build / upload / incremental-update timing.

For each size: native build (rt_builder_add_many), linearisation (rt_builder_desc), full upload
(rt_upload_scene: validation, per-node cull hierarchies, H2D) and, after moving k random entities
(Entity._set_pos + add_entity_to_octree), both re-upload paths: rt_builder_desc + rt_update_scene
(O(scene) on the host) and rt_builder_sync (O(edit)).  One JSON line per measurement.

python tools/scene_timing.py [--tris N ...] [--moves K ...] [--no-gpu]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer.js_amd", "python")]

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, nargs="*", default=[100_000, 1_000_000])
    ap.add_argument("--moves", type=int, nargs="*", default=[1, 10, 100, 1000])
    ap.add_argument("--no-gpu", action="store_true")
    a = ap.parse_args()
    rtamd.load_library()
    ctx = None if a.no_gpu else rtamd.Context(0)
    rng = np.random.default_rng(1)
    for n in a.tris:
        spec = scenes.tri_scene(n, 0.001 * (100_000 / n) ** (1 / 3), 8, n_sph=n // 100, p_mirror=0.25, p_light=0.05)
        t0 = time.perf_counter()
        b = rtamd.Builder.from_spec(spec)
        t1 = time.perf_counter()
        sc = b.arrays()
        t2 = time.perf_counter()
        row = dict(tris=n, entities=len(spec.entities), nodes=int(sc.node_size.size), build_s=t1 - t0,
                   desc_s=t2 - t1)
        if ctx is not None:
            ts = []
            for _ in range(3):
                t3 = time.perf_counter()
                ctx.upload(sc)
                ts.append(time.perf_counter() - t3)
            row["upload_s"] = min(ts)
        print(json.dumps(row), flush=True)
        ne = len(spec.entities) - 1
        for path in ("update", "sync"):
            if ctx is not None and path == "sync":
                st = ctx.sync(b)                                   # first sync: full
            for k in a.moves:
                ids = rng.choice(ne, k, replace=False)
                t3 = time.perf_counter()
                for e in ids:
                    b.move(int(e), rng.uniform(0.05, 0.95, 3))
                t4 = time.perf_counter()
                row = dict(tris=n, path=path, moves=k, move_s=t4 - t3)
                if path == "update":
                    sc = b.arrays()
                    t5 = time.perf_counter()
                    row["desc_s"] = t5 - t4
                    if ctx is not None:
                        st = ctx.update(sc)
                        row.update(update_s=time.perf_counter() - t5, **{"st_" + x: v for x, v in st.as_dict().items()})
                elif ctx is not None:
                    st = ctx.sync(b)
                    row.update(sync_s=time.perf_counter() - t4, **{"st_" + x: v for x, v in st.as_dict().items()})
                print(json.dumps(row), flush=True)
        b.close()


if __name__ == "__main__":
    main()
