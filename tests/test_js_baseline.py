"""The JavaScript restatement of the render path (oracle/js/rt_path.js, bench.py's CPU baseline on
Node) against the C oracle: f32 RGB, hit entity, DFS node id, segment count and status bit-identical,
single-threaded and through the worker_threads split.  CPU only (node v12 in the image)."""
import numpy as np
import pytest

import js_baseline
import oracle
import rtamd
from rtamd import abi, scenes

pytestmark = pytest.mark.skipif(js_baseline.node_binary() is None, reason="node not installed")


def _transmission_spec():
    spec = scenes.small_random(5)
    sh = spec.shades.copy()
    sh["response"][::3] = abi.RT_RESP_TRANSMISSION
    sh["light"][::3] = 0
    ents = spec.entities.copy()
    ents["substance"][::2] = 2          # GLASS
    ents["substance"][1::7] = -1        # undefined substance: refraction from it throws
    return scenes.SceneSpec("transmission", ents, sh)


def _check(spec, W, H, refmax, pixels, tmp_path, threads=1, cam=None):
    cam, cfg = cam or scenes.make_camera(W, H), scenes.make_config(refmax)
    d = str(tmp_path / spec.name)
    js_baseline.export(rtamd.build_scene(spec), cam, cfg, pixels, d)
    info, got = js_baseline.run(d, threads=threads)
    w, root = oracle.build_scene(spec)
    ref = w.trace_frame(root, cam, cfg, pixels=pixels, nthreads=4)
    idx = np.asarray(pixels)
    assert np.array_equal(ref["rgb"].reshape(-1, 3)[idx].view(np.uint32), got["rgb"].view(np.uint32))
    for k in ("hit_entity", "hit_node", "segments", "status"):
        assert np.array_equal(ref[k][idx], got[k]), k
    assert info["segments"] == int(ref["segments"][idx].sum())
    return info, got


@pytest.mark.parametrize("name,W,H,refmax", [("config1", 64, 48, 2), ("small3", 80, 60, 4),
                                             ("small8", 72, 40, 3), ("transmission", 64, 64, 5)])
def test_js_restatement_equals_oracle(name, W, H, refmax, tmp_path):
    spec = {"config1": scenes.config1_spheres, "small3": lambda: scenes.small_random(3),
            "small8": lambda: scenes.small_random(8, n_tri=800, half=0.04),
            "transmission": _transmission_spec}[name]()
    _, got = _check(spec, W, H, refmax, np.arange(W * H), tmp_path)
    assert (got["segments"] > 1).any()      # bounces are exercised


def test_js_restatement_shadow_rays_equal_oracle(tmp_path):
    """Shadow rays (a build extension): the definition restated on the reference's
    object model in JavaScript equals the C oracle's statement bit for bit."""
    spec = scenes.config1_spheres()
    W, H = 64, 48
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(3)
    lights = [((0.25, 0.75, 0.25), (0.6, 0.5, 0.4)), ((0.75, 0.25, 0.75), (0.3, 0.4, 0.9)),
              ((0.5, 0.9, 0.6), (0.2, 0.2, 0.2))]
    d = str(tmp_path / "shadow")
    js_baseline.export(rtamd.build_scene(spec), cam, cfg, np.arange(W * H), d, lights, 0.1)
    _, got = js_baseline.run(d)
    w, root = oracle.build_scene(spec)
    w.set_lights(lights, 0.1)
    ref = w.trace_frame(root, cam, cfg, nthreads=4)
    assert np.array_equal(ref["rgb"].reshape(-1, 3).view(np.uint32), got["rgb"].view(np.uint32))
    w.set_lights([])
    assert not np.array_equal(ref["rgb"], w.trace_frame(root, cam, cfg, nthreads=4)["rgb"])


def test_js_workers_config3_sample(tmp_path):
    """The bench's workload (config 3 scene, 1920x1080) on a pixel sample, split over 3 workers."""
    rng = np.random.default_rng(3)
    pix = np.sort(rng.choice(1920 * 1080, 400, replace=False))
    info, _ = _check(scenes.config3(), 1920, 1080, 2, pix, tmp_path, threads=3)
    assert info["threads"] == 3 and info["pixels"] == 400


def test_js_restatement_post_light_reseat_throws(tmp_path):
    """src/raytracer.ts:276: the walker re-seat after a light hit throws on this scene
    in the JS restatement exactly where the C oracle marks the pixel a fault."""
    spec, cam = scenes.reseat_throw_scene()
    W, H = cam.width, cam.height
    _, got = _check(spec, W, H, 2, np.arange(W * H), tmp_path, cam=cam)
    light = got["hit_entity"] == 0
    assert (got["status"][light] == 2).sum() > 100 and (got["status"][light] == 0).any()
