"""The JavaScript drop-in (raytracer.js_amd/js/raytracer.js): a `Raytracer` with the reference's
constructor and trace_frame() (src/raytracer.ts:281-339) that reads reference-shaped scene objects,
flattens them, and renders through the N-API addon into ExposureBuffer.pixels.

CPU: the flattening reproduces the native builder's arrays bit for bit.
GPU: one frame through node -> N-API -> librt_amd.so equals the oracle.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
import rtamd
from rtamd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNER = os.path.join(ROOT, "tests", "js", "run_dropin.js")
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _dump(tmp_path, spec, cam, cfg):
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


def _node(args, timeout=600):
    r = subprocess.run([NODE] + args, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("name", ["config1", "small3", "config2"])
def test_serialize_matches_native_builder(tmp_path, name):
    spec = {"config1": scenes.config1_spheres, "small3": lambda: scenes.small_random(3),
            "config2": scenes.config2}[name]()
    path = _dump(tmp_path, spec, scenes.make_camera(8, 8), scenes.make_config(2))
    out = _node([RUNNER, path, str(tmp_path / "out"), "--serialize-only"])
    assert "serialize ok" in out


EDIT_OPS = {
    "move_root": ("config1", [{"op": "move", "entity": 0, "pos": [0.5, 0.5, 0.8], "depth": 3}]),
    "move_new_nodes": ("small4", [{"op": "move", "entity": 9,
                                    "pos": [0.22770041975507802, 0.5219043192384103, 0.2345159569779426], "depth": 5}]),
    "many": ("small4", [{"op": "move", "entity": 9, "pos": [0.22770041975507802, 0.5219043192384103, 0.2345159569779426], "depth": 5},
                        {"op": "move", "entity": 13, "pos": [0.8287902268064543, 0.2703745559931393, 0.7072929461731522], "depth": 5},
                        {"op": "add_sphere", "pos": [0.7044694202017586, 0.29964738052273826, 0.18759090183548752], "d": 0.04, "depth": 6, "like": 5},
                        {"op": "add_sphere", "pos": [0.31, 0.62, 0.9], "d": 0.01, "depth": 7, "like": 2},
                        {"op": "shade", "entity": 3, "like": 1}, {"op": "substance", "entity": 7, "like": 1},
                        {"op": "move", "entity": 5, "pos": [0.5, 0.5, 0.5], "depth": 5}]),
    "config2_moves": ("config2", [{"op": "shade", "entity": 10, "like": 20}]),
    # a sphere joins a box-only scene through the journal, then moves by its own _set_pos (which
    # overrides the boxes' one): the second edit must see it
    "new_class": ("boxes", [{"op": "add_sphere", "pos": [0.41, 0.37, 0.52], "d": 0.03, "depth": 6, "like": 0},
                            {"op": "sync"}, {"op": "setpos", "entity": 11, "pos": [0.43, 0.36, 0.52]}]),
}


@pytest.mark.parametrize("name", sorted(EDIT_OPS))
def test_edit_journal_equals_fresh_linearisation(tmp_path, name):
    """CPU: the rt_edit_desc that the drop-in's journal builds, applied to the first linearisation as
    rt_apply_edit applies it (records, sets, substances, DFS ids and shift), equals a fresh
    serialize_scene of the edited tree (tests/js/check_edit.js)."""
    scene, ops = EDIT_OPS[name]
    spec = {"config1": scenes.config1_spheres, "small4": lambda: scenes.small_random(4), "config2": scenes.config2,
            "boxes": lambda: scenes.small_random(4, n_tri=0, n_sph=0, n_box=10)}[scene]()
    path = _dump(tmp_path, spec, scenes.make_camera(8, 8), scenes.make_config(2))
    (tmp_path / "ops.json").write_text(json.dumps(ops))
    out = _node([os.path.join(ROOT, "tests", "js", "check_edit.js"), path, str(tmp_path / "ops.json")])
    assert "edit ok" in out, out


def test_journal_bounds_itself(tmp_path):
    """CPU: a journal past its cap (a Raytracer dropped without close()) forgets its notes, marks
    itself over (the next sync re-reads the scene) and is skipped by later mutator calls; a live
    journal keeps noting (tests/js/check_journal_cap.js)."""
    spec = scenes.small_random(4)
    path = _dump(tmp_path, spec, scenes.make_camera(8, 8), scenes.make_config(2))
    out = _node([os.path.join(ROOT, "tests", "js", "check_journal_cap.js"), path])
    assert "journal cap ok" in out, out


def test_addon_loads_and_fails_loudly_without_gpu():
    """The addon loads; with no GPU create() throws RT_E_NODEVICE (never a silent CPU path)."""
    js = ("const rt=require(%r);const a=rt.load_addon();"
          "if(a.abiVersion()!==5)throw Error('abi');"
          "try{a.create(0);console.log('GPU')}catch(e){console.log(e.code)}"
          "try{a.create([0,0],8);console.log('GPU')}catch(e){console.log(e.code)}"
          "try{a.create([]);console.log('empty accepted')}catch(e){console.log(e.code)}") % os.path.join(ROOT, "raytracer.js_amd", "js", "raytracer.js")
    out = _node(["-e", js]).split()
    assert out[0] in ("GPU", "RT_E_NODEVICE")
    assert out[1] in ("GPU", "RT_E_NODEVICE")
    assert out[2] == "RT_E_INVALID"


def _textured_open(seed):
    s = scenes.small_random(seed, n_sph=80)
    s = scenes.SceneSpec(s.name, s.entities[:-1], s.shades, s.substances, s.root_pos, s.root_size)   # no room box
    return scenes.texture(s, [scenes.test_image(64, 32, 1), scenes.test_image(33, 17, 2)], every=2)


@pytest.mark.gpu
@pytest.mark.parametrize("name,wh,refmax,devices", [("config1", (256, 256), 2, None), ("small4", (200, 150), 3, None),
                                                    ("small4_rough", (200, 150), 4, None),
                                                    ("small5_tex", (160, 120), 3, None),
                                                    ("small4", (200, 150), 3, "0,0,0"),
                                                    ("small4_rough", (200, 150), 4, "0,0")])
def test_dropin_frame_equals_oracle(tmp_path, name, wh, refmax, devices):
    """small4_rough: rough mirrors through options.scatter = 'counter' (RT_SCATTER_COUNTER);
    small5_tex: loaded ImageTextures on entities and the SkySphere; devices: the multi-device context
    (options.devices; parts on the one GPU of the test box, gathered by device copies)."""
    spec = {"config1": scenes.config1_spheres, "small4": lambda: scenes.small_random(4),
            "small4_rough": lambda: scenes.roughen(scenes.small_random(4, p_mirror=0.5)),
            "small5_tex": lambda: _textured_open(5)}[name]()
    seed = 123456789012345 if name.endswith("rough") else None
    cam = scenes.make_camera(*wh)
    cfg = scenes.make_config(refmax, scatter_seed=seed, sky_image=2 if name.endswith("tex") else 0)
    path = _dump(tmp_path, spec, cam, cfg)
    _node([RUNNER, path, str(tmp_path / "out")] + (["--scatter", str(seed)] if seed else []) +
          (["--devices", devices] if devices else []))
    P = wh[0] * wh[1]
    rgb = np.fromfile(tmp_path / "out.rgb", dtype=np.float32)
    ent = np.fromfile(tmp_path / "out.ent", dtype=np.int32)
    node = np.fromfile(tmp_path / "out.node", dtype=np.int32)
    status = np.fromfile(tmp_path / "out.status", dtype=np.uint8)
    assert rgb.size == 3 * P and ent.size == P
    w, root = oracle.build_scene(spec)
    ref = w.trace_frame(root, cam, cfg, nthreads=8)
    assert np.abs(rgb.astype(np.float64) - ref["rgb"]).max() <= 1e-4
    assert np.array_equal(rgb.view(np.uint32), ref["rgb"].view(np.uint32))
    assert np.array_equal(ent, ref["hit_entity"])
    assert np.array_equal(node, ref["hit_node"])
    assert np.array_equal(status, ref["status"])
    stats = json.loads((tmp_path / "out.json").read_text())["stats"]
    assert stats["segments"] == ref["counters"]["segments"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,wh,band_min", [("config1", (256, 256), None), ("small4", (200, 150), "0"),
                                              ("config1", (256, 256), "0"), ("small4_rough", (200, 150), "0")])
def test_dropin_default_options_frame_equals_oracle(tmp_path, name, wh, band_min):
    """The drop-in as a host calls it: trace_frame() with options {} (no ids, no counters), i.e. the
    split passes without the counting kernel, and with RT_BAND_MIN=0 the frame as row bands on their
    own streams (the path 1080p-and-up frames take).  Pixels equal the oracle bit for bit."""
    spec = {"config1": scenes.config1_spheres, "small4": lambda: scenes.small_random(4),
            "small4_rough": lambda: scenes.roughen(scenes.small_random(4, p_mirror=0.5))}[name]()
    seed = 123456789012345 if name.endswith("rough") else None
    cam = scenes.make_camera(*wh)
    cfg = scenes.make_config(3, scatter_seed=seed)
    path = _dump(tmp_path, spec, cam, cfg)
    env = dict(os.environ)
    if band_min is not None:
        env["RT_BAND_MIN"] = band_min
    r = subprocess.run([NODE, RUNNER, path, str(tmp_path / "out"), "--plain"] + (["--scatter", str(seed)] if seed else []),
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert not (tmp_path / "out.ent").exists()
    rgb = np.fromfile(tmp_path / "out.rgb", dtype=np.float32)
    w, root = oracle.build_scene(spec)
    ref = w.trace_frame(root, cam, cfg, nthreads=8)
    assert np.array_equal(rgb.view(np.uint32), ref["rgb"].view(np.uint32))
    st = json.loads((tmp_path / "out.json").read_text())["stats"]
    assert "frame_ms" in st and "segments" not in st, st          # no counters: the split passes ran


@pytest.mark.gpu
@pytest.mark.parametrize("plain", [False, True])
def test_dropin_shadow_rays_equal_oracle(tmp_path, plain):
    """options.lights / options.ambient (shadow rays, a build extension: include/rt.h rt_set_lights)
    through the addon's setLights: the frame equals the oracle's statement of the definition."""
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(160, 120), scenes.make_config(3)
    lights = [((0.25, 0.75, 0.25), (0.6, 0.5, 0.4)), ((0.5, 0.9, 0.6), (0.2, 0.2, 0.2))]
    path = _dump(tmp_path, spec, cam, cfg)
    arg = json.dumps({"lights": [{"pos": list(p), "rgb": list(c)} for p, c in lights], "ambient": 0.15})
    _node([RUNNER, path, str(tmp_path / "out"), "--lights", arg, "--reopen"] + (["--plain"] if plain else []))
    rgb = np.fromfile(tmp_path / "out.rgb", dtype=np.float32)
    # after close(), the next trace_frame()'s new context renders with the same lights
    assert np.array_equal(np.fromfile(tmp_path / "out.3.rgb", dtype=np.float32).view(np.uint32), rgb.view(np.uint32))
    w, root = oracle.build_scene(spec)
    w.set_lights(lights, 0.15)
    ref = w.trace_frame(root, cam, cfg, nthreads=8)
    assert np.array_equal(rgb.view(np.uint32), ref["rgb"].view(np.uint32))
    w.set_lights([])
    assert not np.array_equal(rgb, w.trace_frame(root, cam, cfg, nthreads=8)["rgb"])
    if not plain:
        assert np.array_equal(np.fromfile(tmp_path / "out.ent", dtype=np.int32), ref["hit_entity"])


EDITS = {
    # scene, moved sphere A, entity B takes C's material, A's new position; the second one creates
    # three octree nodes (add_entity_to_octree extends the tree inward)
    "root": (scenes.config1_spheres, 0, 3, 1, (0.5, 0.5, 0.8)),
    "new_nodes": (lambda: scenes.small_random(4), 9, 3, 1, (0.22770041975507802, 0.5219043192384103, 0.2345159569779426)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["journal", "direct"])
@pytest.mark.parametrize("edit", sorted(EDITS))
def test_dropin_scene_edit_updates_incrementally(tmp_path, edit, mode):
    """Edits of the live scene after a first frame.  journal: through the reference's mutators
    (_set_pos + add_entity_to_octree, set_material / set_texture), which the drop-in journals and
    sends as one rt_apply_edit (O(edit): only the touched nodes and sets); direct: the same edit by
    field writes, then invalidate_scene({full: true}) (a full re-read diffed by rt_update_scene).  The
    second frame equals the oracle after the same edits."""
    factory, A, B, Cc, pos = EDITS[edit]
    spec = factory()
    cam, cfg = scenes.make_camera(160, 120), scenes.make_config(3)
    path = _dump(tmp_path, spec, cam, cfg)
    e = spec.entities
    args = [str(A), str(B), str(Cc)] + [repr(float(x)) for x in pos] + [str(int(e[A]["max_in_depth"]))]
    _node([RUNNER, path, str(tmp_path / "out"), "--edit"] + args + (["--direct"] if mode == "direct" else []))
    w, root = oracle.build_scene(spec)
    n0 = len(w.linearize(root)["node_size"])
    w.move_entity(root, A, pos, e[A]["max_in_depth"], e[A]["max_out_depth"])
    w.set_shade(B, e[Cc]["shade"], e[B]["substance"])
    n1 = len(w.linearize(root)["node_size"])
    ref = w.trace_frame(root, cam, cfg, nthreads=8)
    o = str(tmp_path / "out.2")
    rgb = np.fromfile(o + ".rgb", dtype=np.float32)
    assert np.array_equal(rgb.view(np.uint32), ref["rgb"].view(np.uint32))
    assert np.array_equal(np.fromfile(o + ".ent", dtype=np.int32), ref["hit_entity"])
    assert np.array_equal(np.fromfile(o + ".node", dtype=np.int32), ref["hit_node"])
    assert np.array_equal(np.fromfile(o + ".status", dtype=np.uint8), ref["status"])
    upd = json.loads((tmp_path / "out.2.json").read_text())["update"]
    assert upd["full"] == 0, upd
    assert upd["via"] == ("edit" if mode == "journal" else "scene"), upd
    assert upd["new_nodes"] == n1 - n0, (upd, n0, n1)
    if mode == "journal":
        # the moved sphere's old and new node, B's node, and the new nodes
        assert 1 <= upd["dirty_nodes"] <= 3 + (n1 - n0), upd
    if edit == "root":                  # the moved sphere and the re-shaded entity are in view
        first = np.fromfile(tmp_path / "out.rgb", dtype=np.float32)
        assert not np.array_equal(first, rgb)
