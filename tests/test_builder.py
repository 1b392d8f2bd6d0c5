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


# ---- a third restatement, in JavaScript (tests/js/refshape.js add_entity_to_octree) ---------------------
@pytest.mark.parametrize("name", ["config1", "small1", "small4", "config2", "config3"])
def test_js_restatement_builds_the_same_tree(tmp_path, name):
    """The test fixture's add_entity_to_octree (JS, written from src/octree_entity.ts:56-188 apart
    from the native builder and the C oracle), linearised by the drop-in's serialize_scene, equals
    the native builder's tree bit for bit (positions, sizes, parents, children, Set-order lists)."""
    import json
    import os
    import shutil
    import subprocess
    node = shutil.which("node")
    if node is None:
        pytest.skip("node not installed")
    spec = {"config1": scenes.config1_spheres, "small1": lambda: scenes.small_random(1),
            "small4": lambda: scenes.small_random(4), "config2": scenes.config2, "config3": scenes.config3}[name]()
    ents = [dict(type=int(e["type"]), geom=[float(x) for x in e["geom"]], depth=int(e["max_in_depth"]))
            for e in spec.entities]
    assert all(int(e["max_out_depth"]) == 0 for e in spec.entities)
    src = tmp_path / "ents.json"
    src.write_text(json.dumps(dict(root_pos=list(spec.root_pos), root_size=float(spec.root_size), ents=ents)))
    out = tmp_path / "tree.json"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([node, os.path.join(root, "tests", "js", "build_check.js"), str(src), str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    js = json.loads(out.read_text())
    got = rtamd.build_scene(spec)
    n = got.n_nodes
    assert len(js["node_size"]) == n
    assert np.array_equal(np.array(js["node_pos"]).view(np.uint64), got.node_pos.reshape(-1).view(np.uint64))
    assert np.array_equal(np.array(js["node_size"]).view(np.uint64), got.node_size.view(np.uint64))
    assert np.array_equal(np.array(js["node_parent"]), got.node_parent)
    assert np.array_equal(np.array(js["node_child"]).reshape(n, 8), got.node_child.reshape(n, 8))
    assert np.array_equal(np.array(js["node_ent_begin"]), got.node_ent_begin)
    assert np.array_equal(np.array(js["node_ent_count"]), got.node_ent_count)
    assert np.array_equal(np.array(js["list_entity"]), got.list_entity)
