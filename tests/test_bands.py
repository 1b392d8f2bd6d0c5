"""Host-buffer frames as row bands on one GPU (rt_api.hip trace_frame_bands).

rt_trace_frame without counters splits the frame's rows into RT_BANDS bands in the reference's scan
order, traces each on its own stream and copies each into the host buffer as soon as it is done.
The split changes scheduling only: every frame must equal the one-launch frame (RT_BANDS=1) and the
oracle bit for bit, including blends, counter-RNG scatter, odd sizes and the reference's partial
frame after a throw (src/raytracer.ts:318-329).
"""
import numpy as np
import pytest

import oracle
import rtamd
from rtamd import abi, scenes

pytestmark = pytest.mark.gpu

KEYS = ("rgb", "hit_entity", "hit_node", "status")


def _same(a, b):
    for k in KEYS:
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k
    assert a["rc"] == b["rc"]


def _ctx(scene, bands, monkeypatch, order=0):
    monkeypatch.setenv("RT_BANDS", str(bands))
    monkeypatch.setenv("RT_BAND_ORDER", str(order))
    monkeypatch.setenv("RT_BAND_MIN", "0")          # bands at test sizes (the default starts at 2^20 pixels)
    c = rtamd.Context(0)
    c.upload(scene)
    return c


@pytest.fixture(scope="module")
def small3():
    spec = scenes.small_random(3)
    return spec, rtamd.build_scene(spec)


@pytest.mark.parametrize("bands,order", [(2, 0), (3, 1), (4, 3), (8, 0), (8, 3)])
@pytest.mark.parametrize("wh", [(160, 120), (101, 37), (64, 16), (33, 200)])
def test_bands_equal_one_launch(small3, bands, order, wh, monkeypatch):
    """RT_BAND_ORDER 1: level-0 walks chained across bands by events; 2: stream priorities."""
    spec, scene = small3
    cam, cfg = scenes.make_camera(*wh), scenes.make_config(3)
    one = _ctx(scene, 1, monkeypatch)
    many = _ctx(scene, bands, monkeypatch, order)
    try:
        ref = one.trace_frame(cam, cfg, stats=False, allow_fault=True)
        for _ in range(2):                           # the second frame runs with grid hints
            _same(ref, many.trace_frame(cam, cfg, stats=False, allow_fault=True))
        got = many.trace_frame(cam, cfg, ids=False, stats=False, allow_fault=True)
        assert np.array_equal(ref["rgb"].view(np.uint32), got["rgb"].view(np.uint32))
        bcfg = scenes.make_config(3, col_weight=1 / 3)
        old = np.random.default_rng(7).uniform(0, 2, wh[0] * wh[1] * 3).astype(np.float32)
        _same(one.trace_frame(cam, bcfg, rgb=old.copy(), stats=False, allow_fault=True),
              many.trace_frame(cam, bcfg, rgb=old.copy(), stats=False, allow_fault=True))
    finally:
        one.close()
        many.close()


def test_bands_equal_oracle_scatter_and_transmission(monkeypatch):
    """Rough mirrors on the counter RNG (keyed by the full-frame pixel index, so a band's row offset
    must reach it) and glass at refmax 5, 4 bands, against the oracle."""
    spec = scenes.roughen(scenes.small_random(4, p_mirror=0.5))
    cam = scenes.make_camera(200, 150)
    cfg = scenes.make_config(5, scatter_seed=123456789012345)
    c = _ctx(rtamd.build_scene(spec), 4, monkeypatch)
    try:
        got = c.trace_frame(cam, cfg, stats=False, allow_fault=True)
    finally:
        c.close()
    w, root = oracle.build_scene(spec)
    ref = w.trace_frame(root, cam, cfg, nthreads=8)
    assert np.array_equal(ref["rgb"].view(np.uint32), got["rgb"].view(np.uint32))
    assert np.array_equal(ref["hit_entity"], got["hit_entity"]) and np.array_equal(ref["hit_node"], got["hit_node"])
    assert np.array_equal(ref["status"], got["status"])


def _throwing_scene():
    """test_multi_device's scene: glass spheres seen from an undefined substance."""
    spec = scenes.config1_spheres()
    e, sh = spec.entities.copy(), spec.shades.copy()
    sh["response"][:] = abi.RT_RESP_TRANSMISSION
    sh["light"][:] = 0
    e["substance"][:] = 2
    e["substance"][-1] = -1
    return scenes.SceneSpec("throws", e, sh)


@pytest.mark.parametrize("bands", [2, 4, 8])
@pytest.mark.parametrize("ids", [True, False])
def test_bands_keep_the_reference_partial_frame(bands, ids, monkeypatch):
    """A throw inside a band: bands before it in scan order are final, it and later pixels keep the
    previous value, bit for bit with the oracle's aborted frame."""
    spec = _throwing_scene()
    W, H = 96, 72
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(5, default_substance=-1, col_weight=0.5)
    old = np.random.default_rng(5).random(W * H * 3, dtype=np.float32)
    w, root = oracle.build_scene(spec)
    try:
        want = w.trace_frame(root, cam, cfg, rgb=old.copy(), abort=True)
    finally:
        w.close()
    c = _ctx(rtamd.build_scene(spec), bands, monkeypatch)
    try:
        got = c.trace_frame(cam, cfg, rgb=old.copy(), ids=ids, stats=False, allow_fault=True)
    finally:
        c.close()
    assert got["rc"] == abi.RT_E_FAULT
    assert np.array_equal(got["rgb"].view(np.uint32), want["rgb"].view(np.uint32))
    if ids:
        assert np.array_equal(got["status"], want["status"])
