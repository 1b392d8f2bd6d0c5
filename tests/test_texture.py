"""Image textures (include/rt.h rt_image_desc, rt_shade.image, sky_image).

ImageTexture.get_color (src/texture/texture_image.ts:40-63) reads the texel at
((u*W) << 0, (v*H) << 0); uv comes from uv_map_sphere (src/math/uv_mapping.ts:19-25), i.e. from
Math.atan2, for textured spheres (src/entities/entity_sphere.ts:98-101) and the SkySphere
(src/sky/sky_sphere.ts:23-26); boxes and faces map to (0, 0).  V8's Math.atan2 is fdlibm's; the
build restates it (raytracer.js_amd/csrc/rt_jsnum.h for the kernels, oracle/rt_oracle.c for the
oracle) so that texel choices match bit for bit instead of within a tolerance.

Pinning: tests/golden/texture_vectors.json holds V8's atan2 results, uv pairs and texel indices
(tests/golden/gen_texture.js, run by node).  The oracle and the kernels' header (compiled for the
host here) must equal them exactly; GPU frames with textured entities and skies must equal the
oracle's bit for bit.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle
import rtamd
from rtamd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "texture_vectors.json")


def _h(x):
    return np.frombuffer(bytes.fromhex(x), "<f8")[0]


def _bits(x):
    return np.float64(x).view(np.uint64)


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as f:
        return json.load(f)


def _same(a, b):
    return _bits(a) == _bits(b) or (np.isnan(a) and np.isnan(b))


def test_oracle_atan2_matches_v8(gold):
    for y, x, r in gold["atan2"]:
        assert _same(oracle.atan2(_h(y), _h(x)), _h(r)), (y, x)


def test_oracle_uv_and_texels_match_v8(gold):
    for c in gold["uv"]:
        d = [_h(x) for x in c["d_hex"]]
        u, v = oracle.uv_map_sphere(d)
        assert _same(u, _h(c["uv_hex"][0])) and _same(v, _h(c["uv_hex"][1])), c
        for (w, h), t in zip(gold["sizes"], c["texel"]):
            ui, vi = int(np.trunc(u * w)), int(np.trunc(v * h))
            assert (vi * w + ui if -2.220446049250313e-16 <= u <= 1 - 2.220446049250313e-16 and
                    -2.220446049250313e-16 <= v <= 1 - 2.220446049250313e-16 else -1) == t


def test_kernel_header_matches_v8(gold, tmp_path):
    """rt_jsnum.h (the kernels' js_atan2 / uv_map_sphere / texel_index) compiled for the host."""
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include "rt_jsnum.h"
#include <stdio.h>
int main() {
    char kind; unsigned long long a, b, c;
    while (scanf(" %c %llx %llx %llx", &kind, &a, &b, &c) == 4) {
        double x, y, z; memcpy(&x, &a, 8); memcpy(&y, &b, 8); memcpy(&z, &c, 8);
        if (kind == 'a') { double r = rtjs::js_atan2(x, y); unsigned long long o; memcpy(&o, &r, 8); printf("%016llx\n", o); }
        else {
            double u, v; rtjs::uv_map_sphere(x, y, z, u, v);
            unsigned long long ou, ov; memcpy(&ou, &u, 8); memcpy(&ov, &v, 8);
            printf("%016llx %016llx %lld %lld\n", ou, ov, (long long)rtjs::texel_index(u, v, 64, 32),
                   (long long)rtjs::texel_index(u, v, 4096, 2048));
        }
    }
}
''')
    exe = tmp_path / "t"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-I",
                    os.path.join(ROOT, "raytracer.js_amd", "csrc"), str(src), "-o", str(exe)], check=True)

    def le2be(hx):
        return bytes.fromhex(hx)[::-1].hex()
    lines = ["a %s %s 0" % (le2be(y), le2be(x)) for y, x, _ in gold["atan2"]]
    lines += ["u %s %s %s" % tuple(le2be(v) for v in c["d_hex"]) for c in gold["uv"]]
    out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.split("\n")
    k = 0
    for y, x, r in gold["atan2"]:
        got = np.frombuffer(bytes.fromhex(out[k])[::-1], "<f8")[0]
        assert _same(got, _h(r)), (y, x)
        k += 1
    i64, i4096 = gold["sizes"].index([64, 32]), gold["sizes"].index([4096, 2048])
    for c in gold["uv"]:
        hu, hv, t64, t4096 = out[k].split()
        assert _same(np.frombuffer(bytes.fromhex(hu)[::-1], "<f8")[0], _h(c["uv_hex"][0]))
        assert _same(np.frombuffer(bytes.fromhex(hv)[::-1], "<f8")[0], _h(c["uv_hex"][1]))
        assert int(t64) == c["texel"][i64] and int(t4096) == c["texel"][i4096]
        k += 1


def _open(spec):
    """The scene without its enclosing room box (the last entity), so rays reach the sky."""
    return scenes.SceneSpec(spec.name + "_open", spec.entities[:-1], spec.shades, spec.substances, spec.root_pos,
                            spec.root_size, list(spec.images))


def _textured(seed):
    base = _open(scenes.small_random(seed, n_sph=80, p_mirror=0.3))
    imgs = [scenes.test_image(64, 32, 1), scenes.test_image(7, 5, 2), scenes.test_image(1024, 512, 3)]
    return scenes.texture(base, imgs, every=2)


def test_oracle_textures_change_the_frame():
    spec = _textured(3)
    cam = scenes.make_camera(64, 48)
    w, root = oracle.build_scene(spec)
    try:
        a = w.trace_frame(root, cam, scenes.make_config(3), nthreads=4)
        b = w.trace_frame(root, cam, scenes.make_config(3, sky_image=3), nthreads=4)
    finally:
        w.close()
    w2, root2 = oracle.build_scene(_open(scenes.small_random(3, n_sph=80, p_mirror=0.3)))
    try:
        c = w2.trace_frame(root2, cam, scenes.make_config(3), nthreads=4)
    finally:
        w2.close()
    assert not np.array_equal(a["rgb"], c["rgb"])       # textured entities
    assert not np.array_equal(a["rgb"], b["rgb"])       # textured sky
    assert (a["status"] == 0).mean() > 0.9 and (b["status"] == 0).mean() > 0.9


# ---- GPU -----------------------------------------------------------------------------------------------------
def _check(ref, got):
    rr, gg = ref["rgb"].reshape(-1, 3), got["rgb"].reshape(-1, 3)
    assert np.array_equal(rr.view(np.uint32), gg.view(np.uint32)), "%d pixels differ" % int(
        (rr.view(np.uint32) != gg.view(np.uint32)).any(1).sum())
    for k in ("hit_entity", "hit_node", "status"):
        assert np.array_equal(ref[k], got[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("seed,sky", [(3, 0), (5, 3), (8, 1)])
def test_textured_frame_equals_oracle(seed, sky):
    spec = _textured(seed)
    cam, cfg = scenes.make_camera(192, 128), scenes.make_config(4, sky_image=sky)
    w, root = oracle.build_scene(spec)
    ctx = rtamd.Context(0)
    try:
        ref = w.trace_frame(root, cam, cfg, nthreads=8)
        ctx.upload(rtamd.build_scene(spec))
        got = ctx.trace_frame(cam, cfg, stats=False, allow_fault=True)
        _check(ref, got)
        st = ctx.trace_frame(cam, cfg, allow_fault=True)       # the fused stats kernel
        for k in ("rgb", "hit_entity", "hit_node", "status"):
            assert np.array_equal(got[k].view(np.uint8), st[k].view(np.uint8)), k
        with pytest.raises(rtamd.RtError):
            ctx.trace_frame(cam, scenes.make_config(4, sky_image=len(spec.images) + 1))
    finally:
        ctx.close()
        w.close()


@pytest.mark.gpu
def test_texture_edit_through_update():
    """Replacing an image and re-pointing shades travel through rt_update_scene."""
    spec = _textured(4)
    cam, cfg = scenes.make_camera(128, 96), scenes.make_config(3, sky_image=2)
    ctx = rtamd.Context(0)
    try:
        arr = rtamd.build_scene(spec)
        ctx.upload(arr)
        arr.images[1] = scenes.test_image(9, 11, 7)
        arr.shades["image"][arr.shades["image"] == 3] = 1
        st = ctx.update(arr)
        assert st.full == 0 and st.dirty_nodes == 0
        spec2 = scenes.SceneSpec(spec.name, spec.entities, arr.shades, spec.substances, spec.root_pos,
                                 spec.root_size, arr.images)
        w, root = oracle.build_scene(spec2)
        try:
            _check(w.trace_frame(root, cam, cfg, nthreads=8), ctx.trace_frame(cam, cfg, stats=False,
                                                                               allow_fault=True))
        finally:
            w.close()
    finally:
        ctx.close()
