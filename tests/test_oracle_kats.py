"""Pin the oracle (CPU restatement) against the reference's own known-answer tests.

Every case here is a transcription of a reference jest test (tests/golden/reference_kats.json
records file:line).  Pixel colours are not covered by any reference test; see DESIGN.md §Oracle.
"""
import math
import random

import numpy as np
import pytest

import oracle
from rtamd import abi, scenes

EPS = 2.0 ** -52


def test_octree_get_bounds(kats):
    """test/octree.test.ts:3-7 — Octree.get throws outside 0..7."""
    w = oracle.World()
    t = w.tree((0, 0, 0), 1, entity_set=False)
    for n in kats["octree_get_bounds"]["throws_for"]:
        with pytest.raises(IndexError):
            w.get(t, n)
    for n in range(8):
        assert w.get(t, n) is None


def _path(w, root, path):
    t = root
    for n in path:
        t = w.get(t, n)
    return t


def test_node_at_pos_discrete(kats):
    """test/octree-space.test.ts:36-46."""
    k = kats["node_at_pos_discrete"]
    w = oracle.World()
    root = w.tree(k["root"]["pos"], k["root"]["size"], entity_set=False)
    for path in k["subtrees"]:
        w.new_subtree(_path(w, root, path[:-1]), path[-1])
    tree, oc = w.node_at_pos(root, k["point"])
    assert tree == _path(w, root, k["expect_tree_path"])
    assert oc == k["expect_octant"]


def test_node_at_pos_fuzzy():
    """test/octree-space.test.ts:6-34, with a seeded RNG instead of Math.random."""
    w = oracle.World()
    root = w.tree((0, 0, 0), 1, entity_set=False)
    inner = w.new_subtree(root, 0)
    rng = random.Random(1234)
    for _ in range(2000):
        rnd = int(rng.random() * 8)
        p = [rng.uniform(0.5, 1.0) if rnd & (1 << j) else rng.uniform(0.0, 0.5) for j in range(3)]
        expected = root
        if rnd == 0:
            sp = [x * (1 / 0.25) for x in p]
            rnd = (int(sp[0]) << 0) + (int(sp[1]) << 1) + (int(sp[2]) << 2)
            expected = inner
        assert w.node_at_pos(root, p) == (expected, rnd)


def test_entity_placement(kats):
    """test/octree-entity.test.ts:52-63."""
    k = kats["entity_placement"]
    w = oracle.World()
    root = w.tree(k["root"]["pos"], k["root"]["size"], entity_set=True)
    w.set_tables(scenes._shade(mirror=1), scenes.SUBSTANCES)
    for case in k["cases"]:
        eid, fit = w.add_entity(root, abi.RT_ENT_SPHERE, list(case["sphere_pos"]) + [case["diameter"]],
                                0, scenes.SUB_AIR, k["flags"]["max_in_depth"], k["flags"]["max_out_depth"])
        node = _path(w, root, case["expect_tree_path"])
        assert fit == node
        assert w.in_set(node, eid)


def _walk_octants(w, root, pos, d):
    wk = w.walker(root, include_undefined=True)
    return w.walk(wk, pos, d)


def test_walker_one_level(kats):
    """test/octree-space-walker.test.ts:29,31,32,35 (stops minus the final root)."""
    w = oracle.World()
    root = w.tree((0, 0, 0), 1, entity_set=False)
    dirs = {29: (3 / 4, math.sqrt(3) / 4, 0), 31: (5, 3, 2), 32: (1, 1, 1), 35: (2, 1.0, 4)}
    for case in kats["walker_one_level"]["cases"]:
        d = dirs[case["line"]]
        stops = _walk_octants(w, root, case["pos"], d)
        assert stops[-1][1] == root and stops[-1][2] is None        # the root comes last
        assert [s[2] for s in stops[:-1]] == case["expect_octants"], case["line"]


def test_walker_outside_start_yields_root_only(kats):
    """test/octree-space-walker.test.ts:30,33,34 start on/outside the half-open root bounds; the
    reference code (src/octree_space.ts:254-286,330) yields only the root there."""
    w = oracle.World()
    root = w.tree((0, 0, 0), 1, entity_set=False)
    cases = {30: ((1, 1, 0), (-3 / 4, -math.sqrt(3) / 4, 0)),
             33: ((1 + EPS, 1, 1 - EPS), (-1, -1, -1)),
             34: ((1, 1, 1), (-1, -1, -1))}
    for line, (pos, d) in cases.items():
        stops = _walk_octants(w, root, pos, d)
        assert [(s[0], s[2]) for s in stops] == [(root, None)], line


def test_walker_two_level(kats):
    """test/octree-space-walker.test.ts:57-70 — pre/post-order and corner tie-breaks."""
    k = kats["walker_two_level"]
    w = oracle.World()
    root = w.tree((0, 0, 0), 1, entity_set=False)
    ids = {"tree": root}
    for name, n in k["subtrees"].items():
        ids[name] = w.new_subtree(root, n)
    stops = _walk_octants(w, root, k["pos"], k["dir"])
    assert stops[-1][1] == root and stops[-1][2] is None
    got = [(s[1], s[2]) for s in stops[:-1]]
    assert got == [(ids[t], o) for t, o in k["expect"]]


def test_camera_unit_dirs():
    """test/view-camera.test.ts:17-49: |dir|^2 close to 1 on a 100x100 camera (fov pi), for the
    initial state; the rotated states are covered by the JS host tests of Camera itself."""
    cam = scenes.make_camera(100, 100, pos=(0, 0, 0), init_v=None, init_h=None, fov_h=math.pi, fov_v=math.pi)
    xs, ys, d = oracle.camera_scan_literal(cam)
    assert len(xs) == 100 * 100
    assert np.all(np.abs((d * d).sum(1) - 1.0) < 0.005)
    # every pixel exactly once
    assert len(set(zip(xs.tolist(), ys.tolist()))) == 100 * 100


def test_camera_square_literal_equals_rowmajor():
    """For square screens the reference's axis-swapped scan (src/view/camera.ts:242-249) and the
    corrected row-major scan produce identical (x, y, dir) bits."""
    cam = scenes.make_camera(64, 64)
    xs, ys, d = oracle.camera_scan_literal(cam)
    rm = oracle.camera_dirs(cam).reshape(64 * 64, 3)
    idx = ys * 64 + xs
    assert np.array_equal(rm[idx].view(np.uint64), d.view(np.uint64))


def test_camera_generator_order_center_pixel():
    """The first yielded pixel is (W/2, H/2) with dir == norm_fr exactly (iter_h at :225-228)."""
    cam = scenes.make_camera(32, 32)
    xs, ys, d = oracle.camera_scan_literal(cam)
    assert (xs[0], ys[0]) == (16, 16)
    assert tuple(d[0]) == tuple(cam.fr)


@pytest.mark.parametrize("wh", [(8, 8), (9, 9), (16, 16)])
def test_scan_index_is_the_reference_scan_order(wh):
    """oracle.scan_index (the order trace_frame writes pixels, used for the abort at the first
    throwing pixel) equals the literal Camera.get_dir_for_each_pixel order on square screens."""
    cam = scenes.make_camera(*wh)
    xs, ys, _ = oracle.camera_scan_literal(cam)
    idx = oracle.scan_index(cam.width, cam.height)
    assert np.array_equal(idx[ys.astype(np.int64) * cam.width + xs], np.arange(cam.width * cam.height))


def test_abort_at_first_throw_keeps_later_pixels():
    W, H = 6, 4
    old = np.arange(W * H * 3, dtype=np.float32)
    new = -old - 1
    st = np.zeros(W * H, np.uint8)
    st[1 * W + 5] = 2                      # a throw at (5, 1): scan position ry(1)=2 -> 2*6 + rx(5)=2 = 14
    out = oracle.abort_at_first_throw(old, new, st, W, H).reshape(-1, 3)
    idx = oracle.scan_index(W, H)
    assert idx[1 * W + 5] == 14
    assert np.array_equal(out[idx < 14], new.reshape(-1, 3)[idx < 14])
    assert np.array_equal(out[idx >= 14], old.reshape(-1, 3)[idx >= 14])
    assert oracle.abort_at_first_throw(old, new, np.zeros(W * H, np.uint8), W, H) is new
