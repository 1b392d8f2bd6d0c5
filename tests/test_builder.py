"""Host logic: the native scene builder (rt_builder_*, add_entity_to_octree) must produce the same
linearised octree as the oracle's restatement of src/octree_entity.ts:60-188, bit for bit."""
import numpy as np
import pytest

import oracle
import rtamd
from rtamd import abi, scenes


def _compare(spec):
    w, root = oracle.build_scene(spec)
    ref = w.linearize(root)
    got = rtamd.build_scene(spec)
    n = len(ref["node_size"])
    assert got.n_nodes == n
    assert np.array_equal(got.node_pos.reshape(n, 3).view(np.uint64), ref["node_pos"].view(np.uint64))
    assert np.array_equal(got.node_size.view(np.uint64), ref["node_size"].view(np.uint64))
    assert np.array_equal(got.node_parent, ref["node_parent"])
    assert np.array_equal(got.node_child.reshape(n, 8), ref["node_child"])
    assert np.array_equal(got.node_ent_begin, ref["node_ent_begin"])
    assert np.array_equal(got.node_ent_count, ref["node_ent_count"])
    assert np.array_equal(got.list_entity, ref["list_entity"])
    assert len(got.ent_type) == len(spec.entities)
    return got, ref


def test_builder_config1():
    got, ref = _compare(scenes.config1_spheres())
    # 8 level-1 nodes, each holding one sphere; the room box in the root set, added last
    assert got.n_nodes == 9
    assert got.list_entity[got.node_ent_begin[0]] == 8


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_builder_small_random(seed):
    _compare(scenes.small_random(seed))


def test_builder_config2_10k():
    got, _ = _compare(scenes.config2())
    assert got.n_nodes > 1000


def test_builder_sphere_caches():
    """SphereEntity caches: Sphere._dot_pp, Sphere._radius_sq = (d/2)^2, entity._radius_sq = d*d/4."""
    spec = scenes.config1_spheres()
    got = rtamd.build_scene(spec)
    g = got.ent_geom.reshape(-1, 9)[0]
    pos, d = g[:3], g[3]
    assert g[4] == (0.0 + pos[0] * pos[0]) + pos[1] * pos[1] + pos[2] * pos[2]
    assert g[5] == (d / 2) * (d / 2)
    assert g[6] == d * d / 4


def test_builder_entity_placement_kat(kats):
    """test/octree-entity.test.ts:52-63 through the native builder."""
    k = kats["entity_placement"]
    e = np.zeros(2, abi.ENTITY_DTYPE)
    for i, case in enumerate(k["cases"]):
        e[i]["type"] = abi.RT_ENT_SPHERE
        e[i]["geom"][:4] = list(case["sphere_pos"]) + [case["diameter"]]
        e[i]["max_in_depth"], e[i]["max_out_depth"] = 10, 10
    spec = scenes.SceneSpec("kat", e, scenes._shade(mirror=1))
    got = rtamd.build_scene(spec)
    child0 = got.node_child.reshape(-1, 8)[0, 0]
    assert child0 > 0
    assert got.list_entity[got.node_ent_begin[child0]] == 0
    assert got.list_entity[got.node_ent_begin[0]] == 1


def test_builder_outside_growth_reported():
    """An entity outside the root with max_out_depth 0 raises TreeOutsideGrowError (RT_E_TREE)."""
    e = np.zeros(1, abi.ENTITY_DTYPE)
    e[0]["type"] = abi.RT_ENT_SPHERE
    e[0]["geom"][:4] = (1.5, 0.5, 0.5, 0.1)
    spec = scenes.SceneSpec("out", e, scenes._shade())
    with pytest.raises(rtamd.RtError) as ei:
        rtamd.build_scene(spec)
    assert ei.value.code == abi.RT_E_TREE
