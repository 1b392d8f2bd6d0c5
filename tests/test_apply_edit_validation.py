"""rt_apply_edit refuses a malformed edit before it touches the resident scene: new
node slots without a record (value-initialised nodes point at the root, and a walk into one would
cycle), DFS ids and shifts out of range.  The frame after each refusal equals the frame before.
"""
import ctypes as C

import numpy as np
import pytest

import rtamd
from rtamd import abi, scenes

pytestmark = pytest.mark.gpu


def _i32(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(C.POINTER(C.c_int32))


def _node_slots(ctx, scene):
    n_nodes = len(scene.node_size)
    out, p = _i32(np.zeros(n_nodes))
    n = C.c_int32()
    rc = ctx.L.rt_scene_node_slots(ctx.h, p, n_nodes, C.byref(n))
    assert rc == 0, rc
    return n.value


def _edit(ctx, **kw):
    d = abi.rt_edit_desc()
    keep = []
    for k, v in kw.items():
        if k == "rec_cube":
            a = np.ascontiguousarray(v, dtype=np.float64)
            keep.append(a)
            d.rec_cube = a.ctypes.data_as(C.POINTER(C.c_double))
        elif isinstance(v, (list, np.ndarray)):
            a, p = _i32(v)
            keep.append(a)
            setattr(d, k, p)
        else:
            setattr(d, k, v)
    st = abi.rt_update_stats()
    return ctx.L.rt_apply_edit(ctx.h, C.byref(d), C.byref(st))


def test_malformed_edits_are_refused_and_the_scene_stands():
    spec = scenes.small_random(4)
    cam, cfg = scenes.make_camera(64, 48), scenes.make_config(2)
    ctx = rtamd.Context(0)
    try:
        scene = rtamd.build_scene(spec)
        ctx.upload(scene)
        before = ctx.trace_frame(cam, cfg)
        n = _node_slots(ctx, scene)
        ne = len(spec.entities)
        # one new slot and no record for it
        assert _edit(ctx, n_slots=n + 1, n_entities=ne) == abi.RT_E_INVALID
        # a recorded new slot (a leaf under the root) whose DFS id is past the slots
        rec = dict(n_rec=1, rec_slot=[n], rec_cube=[0.0, 0.0, 0.0, 0.5], rec_child=[-1] * 8, rec_up=[0, 0])
        assert _edit(ctx, n_slots=n + 1, n_entities=ne, n_dfs_new=1, dfs_new_slot=[n], dfs_new_val=[n + 1],
                     **rec) == abi.RT_E_INVALID
        assert b"dfs_new_val" in ctx.L.rt_last_error()
        # a shift past the slots, and more shifts than slots
        assert _edit(ctx, n_slots=n, n_entities=ne, n_dfs_shift=1, dfs_shift=[n + 5]) == abi.RT_E_INVALID
        assert _edit(ctx, n_slots=n, n_entities=ne, n_dfs_shift=n + 1, dfs_shift=list(range(n + 1))) == abi.RT_E_INVALID
        after = ctx.trace_frame(cam, cfg)
        assert np.array_equal(before["rgb"].view(np.uint32), after["rgb"].view(np.uint32))
        assert np.array_equal(before["hit_node"], after["hit_node"])
    finally:
        ctx.close()
