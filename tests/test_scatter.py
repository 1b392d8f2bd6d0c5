"""Rough mirrors with the counter-based RNG (include/rt.h RT_SCATTER_COUNTER).

The reference scatters with one sequential FpLcg shared by the whole frame (Ray.scatter_ray,
src/raytracer.ts:121-133,233-235), so its draws depend on the pixel visiting order and no parallel
trace can reproduce them.  RT_SCATTER_COUNTER keeps scatter_ray's algorithm and replaces only the
stream: draw n of the ray through pixel p is a pure function of (seed, p, n).

Pinning: tests/golden/scatter_vectors.json holds V8's results for reflect_ray + scatter_ray
(tests/golden/gen_scatter.js, a plain-JS transliteration run by node, fed the counter stream) — the
oracle's stream and scatter step must equal them bit for bit.  Frames: GPU vs oracle bit-exact
(same bar as tests/test_gpu_parity.py), and independent of scheduling: split = fused, any part
count, any oracle thread count.
"""
import json
import os

import numpy as np
import pytest

import oracle
import rtamd
from rtamd import abi, scenes

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scatter_vectors.json")
SEED = 0x5EED_CAFE_F00D


def _h(x):
    return np.frombuffer(bytes.fromhex(x), "<f8")[0]


def _v(xs):
    return np.array([_h(x) for x in xs])


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as f:
        return json.load(f)


def _py_draw(seed, pixel, n):
    """Pure-Python restatement of the stream (include/rt.h)."""
    M = 2 ** 64 - 1
    z = (seed + pixel * 0x9E3779B97F4A7C15 + (n + 1) * 0xD1B54A32D192ED03) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    z ^= z >> 31
    return (z >> 11) / 2.0 ** 53


def test_counter_stream_matches_v8(gold):
    for d in gold["draws"]:
        seed = int(d["seed"])
        for n, h in enumerate(d["values_hex"]):
            assert oracle.counter_draw(seed, d["pixel"], n) == _h(h) == _py_draw(seed, d["pixel"], n)


def test_oracle_scatter_matches_v8(gold):
    assert len(gold["cases"]) == 64
    for c in gold["cases"]:
        d, n = _v(c["dir_hex"]), _v(c["normal_hex"])
        k = -(0.0 + d[0] * n[0] + d[1] * n[1] + d[2] * n[2]) * 2
        refl = d + n * k                                      # vector.reflection
        assert np.array_equal(refl, _v(c["reflected_hex"]))
        out, draws = oracle.scatter_dir(int(c["seed"]), c["pixel"], 0, n, _h(c["roughness_hex"]), refl)
        assert np.array_equal(out.view(np.uint64), _v(c["out_hex"]).view(np.uint64)), c
        assert draws == c["draws"]
        assert abs(np.linalg.norm(out) - 1) < 1e-12
        assert np.dot(out, n) > -1e-12                        # both blend terms face the normal's side


def test_draw_counter_continues(gold):
    """A second scatter of the same ray continues the stream where the first stopped."""
    c = gold["cases"][3]
    n, r = _v(c["normal_hex"]), _h(c["roughness_hex"])
    a, k = oracle.scatter_dir(1, 2, 0, n, r, _v(c["reflected_hex"]))
    b, k2 = oracle.scatter_dir(1, 2, k, n, r, _v(c["reflected_hex"]))
    assert k2 > k >= 3 and not np.array_equal(a, b)


def _rough_small(seed):
    return scenes.roughen(scenes.small_random(seed, p_mirror=0.5))


def test_oracle_frame_independent_of_schedule():
    """Thread count and the pixel subset change nothing: each pixel's draws are its own."""
    spec = _rough_small(3)
    cam, cfg = scenes.make_camera(64, 48), scenes.make_config(4, scatter_seed=SEED)
    w, root = oracle.build_scene(spec)
    try:
        a = w.trace_frame(root, cam, cfg, nthreads=1)
        b = w.trace_frame(root, cam, cfg, nthreads=5)
        pix = np.arange(7, 64 * 48, 13, dtype=np.int32)
        c = w.trace_frame(root, cam, cfg, pixels=pix, nthreads=3)
    finally:
        w.close()
    for k in ("rgb", "hit_entity", "hit_node", "status"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["rgb"].reshape(-1, 3)[pix].view(np.uint32), c["rgb"].reshape(-1, 3)[pix].view(np.uint32))
    assert (a["status"] == 0).mean() > 0.9


def test_oracle_scatter_changes_image_and_seed_matters():
    spec = _rough_small(4)
    smooth = scenes.small_random(4, p_mirror=0.5)
    cam = scenes.make_camera(48, 48)
    w, root = oracle.build_scene(spec)
    w2, root2 = oracle.build_scene(smooth)
    try:
        a = w.trace_frame(root, cam, scenes.make_config(3, scatter_seed=1), nthreads=4)
        b = w.trace_frame(root, cam, scenes.make_config(3, scatter_seed=2), nthreads=4)
        s = w2.trace_frame(root2, cam, scenes.make_config(3, scatter_seed=1), nthreads=4)
        s0 = w2.trace_frame(root2, cam, scenes.make_config(3), nthreads=4)
        rej = w.trace_frame(root, cam, scenes.make_config(3), nthreads=4)
    finally:
        w.close()
        w2.close()
    assert not np.array_equal(a["rgb"], b["rgb"])
    assert not np.array_equal(a["rgb"], s["rgb"])
    assert np.array_equal(s["rgb"], s0["rgb"])            # roughness 0: the mode changes nothing
    # RT_SCATTER_REJECT: a ray reaching a rough mirror is outside the gate (fault)
    assert (rej["status"] == 2).sum() > (a["status"] == 2).sum()


# ---- GPU -----------------------------------------------------------------------------------------------------
def _frames_equal(a, b):
    for k in ("rgb", "hit_entity", "hit_node", "status"):
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k


def _check_vs_oracle(ref, got):
    rr, gg = ref["rgb"].reshape(-1, 3), got["rgb"].reshape(-1, 3)
    assert np.abs(rr.astype(np.float64) - gg.astype(np.float64)).max() <= 1e-4
    assert np.array_equal(rr.view(np.uint32), gg.view(np.uint32)), "%d pixels differ" % int(
        (rr.view(np.uint32) != gg.view(np.uint32)).any(1).sum())
    for k in ("hit_entity", "hit_node", "status"):
        assert np.array_equal(ref[k], got[k]), k


SPECS = {
    "config1": lambda: scenes.roughen(scenes.config1_spheres()),
    "small3": lambda: _rough_small(3),
    "small8": lambda: scenes.roughen(scenes.small_random(8, n_tri=800, half=0.04, p_mirror=0.6), (0.02, 0.5, 1.0)),
    "config2": lambda: scenes.roughen(scenes.config2()),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SPECS))
def test_rough_frame_equals_oracle(name):
    spec = SPECS[name]()
    cam, cfg = scenes.make_camera(192, 128), scenes.make_config(5, scatter_seed=SEED)
    w, root = oracle.build_scene(spec)
    ctx = rtamd.Context(0)
    try:
        ref = w.trace_frame(root, cam, cfg, nthreads=8)
        ctx.upload(rtamd.build_scene(spec))
        got = ctx.trace_frame(cam, cfg, stats=False, allow_fault=True)
        _check_vs_oracle(ref, got)
        _frames_equal(got, ctx.trace_frame(cam, cfg, allow_fault=True))      # stats build (fused kernel)
        with pytest.raises(rtamd.RtError) as ei:                             # the gate without the stream
            ctx.trace_frame(cam, scenes.make_config(5))
        assert ei.value.code == abi.RT_E_UNSUPPORTED
    finally:
        ctx.close()
        w.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["config1", "small8"])
def test_rough_split_equals_fused(name, monkeypatch):
    """Continuation records carry the draw counter across bounce levels and overflow re-walks."""
    spec = SPECS[name]()
    cam, cfg = scenes.make_camera(320, 200), scenes.make_config(6, scatter_seed=SEED)
    scene = rtamd.build_scene(spec)
    ctxs = []
    try:
        split = rtamd.Context(0)
        ctxs.append(split)
        split.upload(scene)
        a = split.trace_frame(cam, cfg, stats=False, allow_fault=True)
        fused = rtamd.Context(0, flags=abi.RT_CREATE_NO_SPLIT)
        ctxs.append(fused)
        fused.upload(scene)
        _frames_equal(a, fused.trace_frame(cam, cfg, stats=False, allow_fault=True))
        monkeypatch.setenv("RT_CAND_CAP", "1")
        monkeypatch.setenv("RT_CONT_GROUP", "64")
        tiny = rtamd.Context(0)
        ctxs.append(tiny)
        tiny.upload(scene)
        _frames_equal(a, tiny.trace_frame(cam, cfg, stats=False, allow_fault=True))
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,stripe", [(3, 8), (5, 1)])
def test_rough_parts_reassemble(n, stripe):
    """The RNG key is the full-frame pixel index: any stripe partition renders the same frame."""
    import torch
    from rtamd.stripes import StripeGather, source_index
    from rtamd import part_rows
    W, H = 160, 96
    spec = SPECS["small3"]()
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(4, scatter_seed=SEED)
    ctx = rtamd.Context(0)
    try:
        ctx.upload(rtamd.build_scene(spec))
        dev = torch.device("cuda", 0)
        s = torch.cuda.Stream(device=dev)
        full = StripeGather(H, W, 0, 1, stripe, dev)
        ctx.trace_rows_device(cam, cfg, 0, 1, stripe, full.local.data_ptr(), s.cuda_stream)
        src, max_rows = source_index(H, n, stripe)
        stacked = torch.full((n * max_rows, W, 3), float("nan"), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()                    # the fills run on torch's stream, the frames on `s`
        for p in range(n):
            rows, _ = ctx.trace_rows_device(cam, cfg, p, n, stripe, stacked[p * max_rows].data_ptr(), s.cuda_stream)
            assert rows == len(part_rows(H, p, n, stripe))
        s.synchronize()
        got = torch.index_select(stacked, 0, torch.from_numpy(src).to(dev)).cpu().numpy()
        ref = full.local[:H].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        w, root = oracle.build_scene(spec)
        try:
            o = w.trace_frame(root, cam, cfg, nthreads=8)["rgb"].reshape(H, W, 3)
        finally:
            w.close()
        assert np.array_equal(ref.view(np.uint32), o.view(np.uint32))
    finally:
        ctx.close()
