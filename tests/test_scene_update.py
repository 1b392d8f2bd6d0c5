"""Scene edits and incremental re-upload (include/rt.h rt_update_scene,
rt_builder_move / rt_builder_set_shade).

The reference edits a live scene with add_entity_to_octree (src/octree_entity.ts:174-188), moves
an entity with Entity._set_pos + add_entity_to_octree, which re-files it through
Entity.set_octree (src/entity.ts:50-56: Set.delete, then Set.add, so the entity goes to the END of
its new node's Set order even when the node is the same), and re-materials it with
set_material / set_texture / set_substance.

CPU: the native builder and the oracle apply the same edit sequence to identical trees (Set order
included).  GPU: after each edit, rt_update_scene's frame equals a fresh rt_upload_scene of the
same scene and the oracle's frame bit for bit, and the update touched only the edited nodes.
"""
import numpy as np
import pytest

import oracle
import rtamd
from rtamd import abi, scenes

LIN_KEYS = ("node_pos", "node_size", "node_parent", "node_child", "node_ent_begin", "node_ent_count", "list_entity")


def _lin_equal(w, root, arr):
    ref = w.linearize(root)
    for k in LIN_KEYS:
        assert np.array_equal(np.ravel(ref[k]), np.ravel(getattr(arr, k))), k


def _entity(etype, geom, shade, sub=-1, depth=6):
    e = np.zeros(1, abi.ENTITY_DTYPE)
    e["type"], e["shade"], e["substance"] = etype, shade, sub
    e["max_in_depth"], e["max_out_depth"] = depth, 0
    e["geom"][0, :len(geom)] = geom
    return e


def _edits(spec, seed):
    """A deterministic edit script over `spec`: moves (to far cells, within the same cell), added
    spheres / triangles, and shade / substance changes."""
    st = scenes.Stream(seed)
    ne = len(spec.entities) - 1                  # the room box (last) never moves
    ops = []
    for k in range(12):
        u = st.take(4)
        eid = int(u[0] * ne)
        kind = k % 4
        if kind == 0:
            ops.append(("move", eid, tuple(0.1 + 0.8 * u[1:4])))
        elif kind == 1:
            g = spec.entities[eid]["geom"]
            t = spec.entities[eid]["type"]
            c = g[:3] if t != abi.RT_ENT_FACE else (g[0:3] + g[3:6] + g[6:9]) / 3
            ops.append(("move", eid, tuple(c + (u[1:4] - 0.5) * 1e-4)))       # usually the same node
        elif kind == 2:
            c = 0.1 + 0.8 * u[1:4]
            if k % 8 == 2:
                ops.append(("add", _entity(abi.RT_ENT_SPHERE, [*c, 0.01 + 0.02 * u[0]], eid % len(spec.shades))))
            else:
                v = np.concatenate([c, c + [0.02, 0, 0.001], c + [0, 0.02, 0.003]])
                ops.append(("add", _entity(abi.RT_ENT_FACE, v, eid % len(spec.shades))))
        else:
            ops.append(("shade", eid, (eid * 7 + k) % len(spec.shades), -1 if k % 2 else 1))
    return ops


class Pair:
    """The same scene as a native builder and an oracle World; edits go to both."""

    def __init__(self, spec):
        self.b = rtamd.Builder.from_spec(spec)
        self.w, self.root = oracle.build_scene(spec)
        self.ents = spec.entities.copy()            # AddEntityToOctreeFlags per entity id

    def apply(self, *ops):
        for op in ops:
            if op[0] == "move":
                _, eid, pos = op
                self.b.move(eid, pos)
                e = self.ents[eid]
                self.w.move_entity(self.root, eid, pos, e["max_in_depth"], e["max_out_depth"])
            elif op[0] == "add":
                self.b.add(op[1])
                self.ents = np.concatenate([self.ents, op[1]])
                self.w.add_entities(self.root, op[1])
            else:
                _, eid, shade, sub = op
                self.b.set_shade(eid, shade, sub)
                self.w.set_shade(eid, shade, sub)

    def close(self):
        self.b.close()
        self.w.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_builder_edits_match_oracle(seed):
    spec = scenes.small_random(seed)
    p = Pair(spec)
    try:
        _lin_equal(p.w, p.root, p.b.arrays())
        for op in _edits(spec, seed):
            p.apply(op)
            _lin_equal(p.w, p.root, p.b.arrays())
    finally:
        p.close()


def test_move_within_node_goes_to_set_end():
    """Set.delete + Set.add: an entity re-filed into the node it was in moves to the end of its Set."""
    spec = scenes.config1_spheres()                  # 8 spheres, each alone in its own depth-3 node
    p = Pair(spec)
    b = p.b
    try:
        a = b.arrays()
        room = len(spec.entities) - 1
        before = a.list_entity[a.node_ent_begin[0]:a.node_ent_begin[0] + a.node_ent_count[0]].tolist()
        # put sphere 0 at the root (its AABB now straddles the centre) then back: it lands after the room box
        p.apply(("move", 0, (0.5, 0.5, 0.5)))
        a = b.arrays()
        lst = a.list_entity[a.node_ent_begin[0]:a.node_ent_begin[0] + a.node_ent_count[0]].tolist()
        assert lst == before + [0] and room in lst
        p.apply(("move", 0, (0.5, 0.5, 0.5 + 1e-9)))                   # same node again: still last
        p.apply(("move", room, tuple(spec.entities[room]["geom"][:3])))  # room box: now last
        a = b.arrays()
        lst = a.list_entity[a.node_ent_begin[0]:a.node_ent_begin[0] + a.node_ent_count[0]].tolist()
        assert lst[-2:] == [0, room]
        _lin_equal(p.w, p.root, a)
    finally:
        p.close()


# ---- GPU -----------------------------------------------------------------------------------------------------
def _frame(ctx, cam, cfg):
    return ctx.trace_frame(cam, cfg, stats=False, allow_fault=True)


def _same(a, b, keys=("rgb", "hit_entity", "hit_node", "status")):
    for k in keys:
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k


@pytest.mark.gpu
@pytest.mark.parametrize("seed,top", [(1, None), (4, None), (4, "3")])
def test_update_equals_full_upload_and_oracle(seed, top, monkeypatch):
    """top: RT_TOP_LEVELS (the upper levels take the first slots, breadth-first)."""
    if top:
        monkeypatch.setenv("RT_TOP_LEVELS", top)
    spec = scenes.small_random(seed, n_tri=600)
    cam, cfg = scenes.make_camera(160, 120), scenes.make_config(3)
    p = Pair(spec)
    ctx, fresh = rtamd.Context(0), rtamd.Context(0)
    try:
        ctx.upload(p.b.arrays())
        for i, op in enumerate(_edits(spec, seed)):
            p.apply(op)
            arr = p.b.arrays()
            st = ctx.update(arr)
            assert st.full == 0, st.as_dict()
            assert st.dirty_nodes <= 4 and st.bytes < 64 * 1024, st.as_dict()
            got = _frame(ctx, cam, cfg)
            fresh.upload(arr)
            _same(got, _frame(fresh, cam, cfg))
            if i % 4 == 3:
                _same(got, p.w.trace_frame(p.root, cam, cfg, nthreads=8))
    finally:
        ctx.close()
        fresh.close()
        p.close()


@pytest.mark.gpu
def test_update_many_edits_regions_and_new_nodes():
    """Repeated growth of one node's Set (regions move to the pool end), new deeper nodes (slots
    appended, node ids through node_dfs), then a scene that is not an edit (full upload)."""
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(128, 96), scenes.make_config(4)
    p = Pair(spec)
    w, root = p.w, p.root
    ctx = rtamd.Context(0)
    try:
        ctx.upload(p.b.arrays())
        st_all = []
        for k in range(40):
            c = (0.05 + 0.9 * ((k * 0.381966) % 1), 0.1 + 0.02 * (k % 7), 0.3 + 0.01 * k)
            e = _entity(abi.RT_ENT_SPHERE, [*c, 0.004], k % 8, depth=7 if k % 3 else 2)
            p.apply(("add", e))
            st_all.append(ctx.update(p.b.arrays()).as_dict())
        assert all(s["full"] == 0 for s in st_all)
        assert sum(s["new_nodes"] for s in st_all) > 0
        assert sum(s["moved_regions"] for s in st_all) > 0
        got = _frame(ctx, cam, cfg)
        _same(got, w.trace_frame(root, cam, cfg, nthreads=8))
        # the debug walk reports DFS ids although new nodes sit in appended slots
        w.linearize(root)
        wk = w.walker(root, include_undefined=True)
        rng = np.random.default_rng(5)
        for _ in range(50):
            o, d = rng.uniform(0.0, 1.0, 3).tolist(), rng.normal(size=3).tolist()
            ref = [(w.tree_id(pt), -1 if po is None else po) for _, pt, po in w.walk(wk, o, d)]
            assert ctx.debug_walk(o, d, include_undefined=True) == ref
        # a different scene through rt_update_scene: falls back to a full upload
        other = rtamd.build_scene(scenes.small_random(2))
        st = ctx.update(other)
        assert st.full == 1
        fresh = rtamd.Context(0)
        try:
            fresh.upload(other)
            _same(_frame(ctx, cam, cfg), _frame(fresh, cam, cfg))
        finally:
            fresh.close()
    finally:
        ctx.close()
        p.close()


@pytest.mark.gpu
def test_update_shade_table_and_scatter_gate():
    """A shade-table edit (a mirror made rough) travels without touching any node; the rough-mirror
    gate follows the new table."""
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(64, 64), scenes.make_config(3)
    ctx = rtamd.Context(0)
    try:
        arr = rtamd.build_scene(spec)
        ctx.upload(arr)
        sh = arr.shades.copy()
        sh["roughness"][1] = 0.4
        arr2 = rtamd.SceneArrays(**{k: getattr(arr, k) for k in rtamd.SceneArrays.FIELDS if k != "shades"}, shades=sh)
        st = ctx.update(arr2)
        assert st.full == 0 and st.dirty_nodes == 0 and st.bytes < 4096
        with pytest.raises(rtamd.RtError):
            ctx.trace_frame(cam, cfg)
        cfg_c = scenes.make_config(3, scatter_seed=9)
        fresh = rtamd.Context(0)
        try:
            fresh.upload(arr2)
            _same(_frame(ctx, cam, cfg_c), _frame(fresh, cam, cfg_c))
        finally:
            fresh.close()
    finally:
        ctx.close()


# ---- rt_builder_sync: O(edit) re-upload from the builder's journal ---------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("seed,top", [(1, None), (4, None), (1, "2")])
def test_builder_sync_equals_full_upload_and_oracle(seed, top, monkeypatch):
    """rt_builder_sync after each edit of the script: only the edit's nodes travel (no linearisation,
    no diff of the whole scene), and the frame equals a fresh rt_upload_scene of the builder's
    linearised tree and, periodically, the oracle's frame.  top: RT_TOP_LEVELS (the full sync's slots
    are not DFS order; the builder takes them from the store)."""
    if top:
        monkeypatch.setenv("RT_TOP_LEVELS", top)
    spec = scenes.small_random(seed, n_tri=600)
    cam, cfg = scenes.make_camera(160, 120), scenes.make_config(3)
    p = Pair(spec)
    ctx, fresh = rtamd.Context(0), rtamd.Context(0)
    try:
        st = ctx.sync(p.b)
        assert st.full == 1                                   # the first sync uploads in full
        for i, op in enumerate(_edits(spec, seed)):
            p.apply(op)
            st = ctx.sync(p.b)
            assert st.full == 0, st.as_dict()
            assert st.dirty_nodes <= 4 and st.bytes < 64 * 1024, st.as_dict()
            got = _frame(ctx, cam, cfg)
            fresh.upload(p.b.arrays())
            _same(got, _frame(fresh, cam, cfg))
            if i % 4 == 3:
                _same(got, p.w.trace_frame(p.root, cam, cfg, nthreads=8))
    finally:
        ctx.close()
        fresh.close()
        p.close()


@pytest.mark.gpu
def test_builder_sync_new_nodes_shades_and_fallbacks():
    """Growth into new deeper nodes (appended slots, node_dfs renumbered), shade-table edits that arm the
    rough-mirror gate, an rt_upload_scene in between (the next sync is full again), and the debug
    walk's DFS ids."""
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(128, 96), scenes.make_config(4)
    p = Pair(spec)
    w, root = p.w, p.root
    ctx = rtamd.Context(0)
    try:
        assert ctx.sync(p.b).full == 1
        sts = []
        for k in range(40):
            c = (0.05 + 0.9 * ((k * 0.381966) % 1), 0.1 + 0.02 * (k % 7), 0.3 + 0.01 * k)
            p.apply(("add", _entity(abi.RT_ENT_SPHERE, [*c, 0.004], k % 8, depth=7 if k % 3 else 2)))
            if k % 5 == 4:
                p.apply(("move", k, (0.2 + 0.015 * k, 0.6, 0.4)), ("shade", k + 1, (k + 3) % 8, 1))
            sts.append(ctx.sync(p.b).as_dict())
        assert all(s["full"] == 0 for s in sts)
        assert sum(s["new_nodes"] for s in sts) > 0 and sum(s["moved_regions"] for s in sts) > 0
        got = _frame(ctx, cam, cfg)
        _same(got, w.trace_frame(root, cam, cfg, nthreads=8))
        w.linearize(root)
        wk = w.walker(root, include_undefined=True)
        rng = np.random.default_rng(5)
        for _ in range(40):
            o, d = rng.uniform(0.0, 1.0, 3).tolist(), rng.normal(size=3).tolist()
            ref = [(w.tree_id(pt), -1 if po is None else po) for _, pt, po in w.walk(wk, o, d)]
            assert ctx.debug_walk(o, d, include_undefined=True) == ref
        # a rough mirror in the shade table: the gate follows it without a full upload
        p.b.shades = p.b.shades.copy()
        p.b.shades["roughness"][1] = 0.4
        st = ctx.sync(p.b)
        assert st.full == 0 and st.dirty_nodes == 0
        with pytest.raises(rtamd.RtError):
            ctx.trace_frame(cam, cfg)
        # another upload to the context: the builder's journal no longer applies
        ctx.upload(rtamd.build_scene(scenes.small_random(2)))
        assert ctx.sync(p.b).full == 1
        fresh = rtamd.Context(0)
        try:
            fresh.upload(p.b.arrays())
            cfg_c = scenes.make_config(4, scatter_seed=3)
            _same(_frame(ctx, cam, cfg_c), _frame(fresh, cam, cfg_c))
        finally:
            fresh.close()
    finally:
        ctx.close()
        p.close()


@pytest.mark.gpu
def test_full_sync_waits_for_a_frame_in_flight():
    """A full upload (here: the first rt_builder_sync after rt_upload_scene) overwrites the resident
    scene arrays in place.  A frame launched just before it with rt_trace_frame_device on a caller
    stream must still see the old scene: the upload synchronises the context's devices first."""
    import torch
    old_spec, new_spec = scenes.config2(), scenes.small_random(3)
    cam, cfg = scenes.make_camera(1920, 1080), scenes.make_config(1)
    ctx = rtamd.Context(0)
    b = rtamd.Builder.from_spec(new_spec)
    try:
        ctx.upload(rtamd.build_scene(old_spec))
        s = torch.cuda.Stream()
        want = torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda")
        ctx.trace_frame_device(cam, cfg, want.data_ptr(), s.cuda_stream)
        s.synchronize()
        for _ in range(3):
            got = torch.zeros_like(want)
            torch.cuda.synchronize()
            ctx.trace_frame_device(cam, cfg, got.data_ptr(), s.cuda_stream)   # in flight ...
            st = ctx.sync(b)                                                   # ... while the scene changes
            s.synchronize()
            assert st.full == 1
            assert torch.equal(got.view(torch.int32), want.view(torch.int32))
            ctx.upload(rtamd.build_scene(old_spec))                            # back for the next round
    finally:
        ctx.close()
        b.close()
