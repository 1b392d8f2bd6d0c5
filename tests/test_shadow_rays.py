"""Shadow rays: a BUILD EXTENSION (rt_set_lights, include/rt.h).  The reference samples
no lights (src/raytracer.ts:168-277), so no reference output pins this: the oracle's statement of the
frozen definition (oracle/rt_oracle.c shadow_factor) is the parity target, and the CPU tests below
check that statement's properties.  Lights off (the default) is the reference bit for bit.
"""
import numpy as np
import pytest

import oracle
import rtamd
from rtamd import abi, scenes

# config 1's two light spheres (k = 2, 5) and a light outside every entity
LIGHTS = [((0.25, 0.75, 0.25), (0.6, 0.5, 0.4)), ((0.75, 0.25, 0.75), (0.3, 0.4, 0.9)),
          ((0.5, 0.9, 0.6), (0.2, 0.2, 0.2))]


def _oracle_frame(spec, cam, cfg, lights=None, ambient=0.0):
    w, root = oracle.build_scene(spec)
    if lights is not None:
        w.set_lights(lights, ambient)
    return w.trace_frame(root, cam, cfg, nthreads=8)


def test_oracle_lights_off_is_the_reference():
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(48, 32), scenes.make_config(3)
    ref = _oracle_frame(spec, cam, cfg)
    w, root = oracle.build_scene(spec)
    w.set_lights(LIGHTS, 0.5)
    w.set_lights([])                                     # back off
    got = w.trace_frame(root, cam, cfg, nthreads=8)
    assert np.array_equal(ref["rgb"].view(np.uint32), got["rgb"].view(np.uint32))


def test_oracle_dark_lights_and_unit_ambient_are_the_reference():
    """s = 1 + 0*k = 1 exactly: every matte pixel keeps the reference's colour."""
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(48, 32), scenes.make_config(3)
    ref = _oracle_frame(spec, cam, cfg)
    dark = [(p, (0.0, 0.0, 0.0)) for p, _ in LIGHTS]
    got = _oracle_frame(spec, cam, cfg, dark, 1.0)
    assert np.array_equal(ref["rgb"].view(np.uint32), got["rgb"].view(np.uint32))
    assert np.array_equal(ref["hit_entity"], got["hit_entity"])
    assert np.array_equal(ref["status"], got["status"])


def test_oracle_a_light_listed_twice_doubles_its_term():
    """ambient 0: s = 0 + x + x = 2x exactly, and col*(2x) = 2*(col*x) in binary64 and after the f32
    store, so every pixel of the two-light frame is exactly twice the one-light frame's."""
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(48, 32), scenes.make_config(3)
    one = _oracle_frame(spec, cam, cfg, LIGHTS[:1], 0.0)
    two = _oracle_frame(spec, cam, cfg, LIGHTS[:1] * 2, 0.0)
    lit = one["rgb"] != 0
    assert lit.any(), "no pixel receives the light"
    ref = _oracle_frame(spec, cam, cfg)
    matte = (one["rgb"] != ref["rgb"]).reshape(-1, 3).any(1)        # pixels the lights changed
    m3 = np.repeat(matte, 3)
    assert np.array_equal(two["rgb"][m3], 2 * one["rgb"][m3])
    assert np.array_equal(two["rgb"][~m3], one["rgb"][~m3])


def test_oracle_a_light_outside_the_room_only_leaves_ambient():
    """A light outside the room box (matte, not a light) is blocked from every surface inside it: the
    frame equals the dark-light frame of the same ambient."""
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(48, 32), scenes.make_config(3)
    outside = [((1.6, 1.7, 1.8), (5.0, 5.0, 5.0))]
    got = _oracle_frame(spec, cam, cfg, outside, 0.25)
    dark = _oracle_frame(spec, cam, cfg, [((1.6, 1.7, 1.8), (0.0, 0.0, 0.0))], 0.25)
    assert np.array_equal(got["rgb"].view(np.uint32), dark["rgb"].view(np.uint32))


def test_oracle_shadow_rays_change_matte_pixels_only():
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(48, 32), scenes.make_config(3)
    ref = _oracle_frame(spec, cam, cfg)
    got = _oracle_frame(spec, cam, cfg, LIGHTS, 0.1)
    changed = (got["rgb"] != ref["rgb"]).reshape(-1, 3).any(1)
    assert changed.any()
    assert np.array_equal(ref["hit_entity"], got["hit_entity"])
    assert np.array_equal(ref["hit_node"], got["hit_node"])
    # a pixel whose colour is the sky's or a light's (not matte) is untouched
    assert not changed[ref["hit_entity"] < 0].any()


def test_light_arrays_bounded():
    with pytest.raises(ValueError):
        abi.lights_array(LIGHTS * 2)


# ---- GPU parity against the oracle's statement ----------------------------------------------------

SPLIT = {"RT_FUSE_MAX": "0", "RT_FUSE_LIST": "0"}      # every frame on the split path (k_shadow)

SHADOW_CASES = [
    # config 1 (few entities: the fused kernel, shadow rays inline) and forced onto the split path
    ("config1", (160, 120), 3, LIGHTS, 0.1, {}),
    ("config1", (160, 120), 3, LIGHTS, 0.1, {"env": SPLIT}),
    # small4: the split path, matte ends deferred to k_shadow from k_shade and the segmented levels
    ("small4", (128, 96), 4, LIGHTS[1:], 0.0, {}),
    ("small4", (128, 96), 4, LIGHTS, 0.3, {"stats": True}),                 # the fused counting kernel
    ("small4", (96, 64), 3, LIGHTS[:2], 0.2, {"devices": [0, 0]}),
    ("small4", (128, 96), 4, LIGHTS, 0.1, {"env": dict(SPLIT, RT_CAND_CAP="2")}),   # overflow: k_cont defers
    ("small4", (128, 96), 4, LIGHTS, 0.1, {"env": dict(SPLIT, RT_SEG="1")}),        # unsegmented levels
    ("config1", (96, 64), 3, LIGHTS, 0.0, {"blend": 0.25}),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,wh,refmax,lights,ambient,opt", SHADOW_CASES)
def test_shadow_rays_equal_oracle(monkeypatch, name, wh, refmax, lights, ambient, opt):
    for k, v in opt.get("env", {}).items():
        monkeypatch.setenv(k, v)                      # read at rt_create
    spec = {"config1": scenes.config1_spheres, "small4": lambda: scenes.small_random(4)}[name]()
    cam = scenes.make_camera(*wh)
    blend = opt.get("blend")
    cfg = scenes.make_config(refmax, col_weight=blend if blend else 1.0)
    P = wh[0] * wh[1]
    rng = np.random.default_rng(5)
    old = rng.random(P * 3).astype(np.float32) if blend else np.zeros(P * 3, np.float32)
    w, root = oracle.build_scene(spec)
    w.set_lights(lights, ambient)
    ref = w.trace_frame(root, cam, cfg, rgb=old.copy(), nthreads=8)
    ctx = rtamd.Context(0, devices=opt.get("devices"))
    try:
        ctx.upload(rtamd.build_scene(spec))
        ctx.set_lights(lights, ambient)
        got = ctx.trace_frame(cam, cfg, rgb=old.copy(), stats=opt.get("stats", False))
        assert np.array_equal(ref["rgb"].view(np.uint32), got["rgb"].view(np.uint32)), \
            "%d pixels differ" % int((ref["rgb"] != got["rgb"]).sum())
        assert np.array_equal(ref["hit_entity"], got["hit_entity"])
        assert np.array_equal(ref["hit_node"], got["hit_node"])
        assert np.array_equal(ref["status"], got["status"])
        # lights off again: the reference frame (the split path) on the same context
        ctx.set_lights([])
        plain = ctx.trace_frame(cam, cfg, rgb=old.copy())
        w.set_lights([])
        ref0 = w.trace_frame(root, cam, cfg, rgb=old.copy(), nthreads=8)
        assert np.array_equal(ref0["rgb"].view(np.uint32), plain["rgb"].view(np.uint32))
    finally:
        ctx.close()


@pytest.mark.gpu
def test_set_lights_rejects_bad_arguments():
    ctx = rtamd.Context(0)
    try:
        arr = abi.lights_array(LIGHTS)
        assert ctx.L.rt_set_lights(ctx.h, arr, abi.RT_MAX_LIGHTS + 1, 0.0) == abi.RT_E_INVALID
        assert ctx.L.rt_set_lights(ctx.h, arr, -1, 0.0) == abi.RT_E_INVALID
        assert ctx.L.rt_set_lights(ctx.h, None, 1, 0.0) == abi.RT_E_INVALID
        assert ctx.L.rt_set_lights(ctx.h, arr, 1, float("nan")) == abi.RT_E_INVALID
        arr[0].pos[1] = float("inf")
        assert ctx.L.rt_set_lights(ctx.h, arr, 1, 0.0) == abi.RT_E_INVALID
        assert ctx.L.rt_set_lights(ctx.h, None, 0, 0.0) == 0
    finally:
        ctx.close()
