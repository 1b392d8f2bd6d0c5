"""Device-resident ExposureBuffer consumers: luminance statistics, the
tone-mapper dynamic range and the RGBA8 canvas image (src/view/exposure_buffer.ts:53-158,
src/view/tone_mapping.ts:22-80, src/view/screen_canvas.ts:45-55,92-94), and progressive
accumulation with rt_trace_rows_device.

Pinning: tests/golden/exposure_vectors.json holds V8's own results (tests/golden/gen_exposure.js,
a plain-JS transliteration run by node) — the oracle must equal them bit for bit.
Tolerances: the device sums the statistics in a fixed tree order, the reference sequentially.
Every summand is nonnegative, so the reference's recursive sum is within (n-1)*2^-53 (relative) of
the exact sum and the tree sum within log2(n)*2^-53: mean / variance / absdev must agree to a
relative n * 2^-52.  Everything else (ranges from identical statistics, RGBA8, accumulated RGB)
is bit-exact.
"""
import json
import os
import struct

import numpy as np
import pytest

import oracle
import rtamd
from rtamd import abi, scenes

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "exposure_vectors.json")


def stats_rtol(n):
    return max(n, 1) * 2.0 ** -52


def _h2d(h):
    return struct.unpack("<d", bytes.fromhex(h))[0]


def _same(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64)) or np.array_equal(a, b, equal_nan=True)


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as f:
        d = json.load(f)
    for c in d["cases"]:
        c["rgb"] = np.frombuffer(bytes.fromhex(c["rgb_f32_hex"]), np.float32).copy()
        c["stats"] = [_h2d(x) for x in c["stats_hex"]]
        c["ranges"] = [[_h2d(x) for x in r] for r in c["ranges_hex"]]
    return d["cases"]


def test_oracle_matches_v8_goldens(gold):
    for c in gold:
        assert _same(oracle.exposure_stats(c["rgb"]), c["stats"]), c["name"]
        for mode in range(3):
            assert _same(oracle.tonemap_range(mode, np.array(c["stats"])), c["ranges"][mode]), (c["name"], mode)
        lo, hi = c["ranges"][1]
        assert np.array_equal(oracle.tonemap(c["rgb"], lo, hi), np.array(c["rgba_stddev"], np.uint8)), c["name"]
        assert np.array_equal(oracle.tonemap(c["rgb"], 0, 1), np.array(c["rgba_identity"], np.uint8)), c["name"]


def test_library_tonemap_range_matches_goldens(gold):
    """rt_tonemap_range is host arithmetic in librt_amd.so: callable without a GPU."""
    for c in gold:
        st = abi.rt_exposure_stats(*c["stats"])
        for mode in range(3):
            assert _same(rtamd.tonemap_range(mode, st), c["ranges"][mode]), (c["name"], mode)
    with pytest.raises(rtamd.RtError):
        rtamd.tonemap_range(7, abi.rt_exposure_stats(1, 1, 1))


def test_tonemap_range_dynamic_range_shift():
    """dynamic_coef = 1 << dynamic_range uses ToInt32 shift semantics (count masked to 5 bits)."""
    st = abi.rt_exposure_stats(0.5, 0.04, 0.1)
    for dr in (0, 1, 8, 12, 31, 32, 40):
        assert _same(rtamd.tonemap_range(1, st, dr), oracle.tonemap_range(1, [0.5, 0.04, 0.1], dr))


# ---- GPU -----------------------------------------------------------------------------------------------------
def _stats_close(got, ref, n):
    for g, r in zip(got, ref):
        if np.isnan(r) or np.isinf(r):
            assert _same([g], [r])
        else:
            assert abs(g - r) <= stats_rtol(n) * max(abs(r), 1e-300), (g, r, n)


@pytest.mark.gpu
def test_device_stats_and_tonemap_goldens(gold):
    import torch
    ctx = rtamd.Context(0)
    try:
        for c in gold:
            n = c["n_pixels"]
            d = torch.from_numpy(c["rgb"]).cuda()
            torch.cuda.synchronize()
            st = ctx.exposure_stats_device(d.data_ptr(), n)
            _stats_close([st.mean, st.variance, st.absdev], c["stats"], n)
            for key, (lo, hi) in (("rgba_stddev", c["ranges"][1]), ("rgba_identity", (0.0, 1.0))):
                out = torch.zeros(4 * n, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()            # the fill runs on torch's stream, the kernel on the context's
                ctx.tonemap_device(d.data_ptr(), n, lo, hi, out.data_ptr())
                torch.cuda.synchronize()
                assert np.array_equal(out.cpu().numpy(), np.array(c[key], np.uint8)), (c["name"], key)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_progressive_exposure_device_resident():
    """Three frames blended on the device (col_weight 1, 1/2, 1/3 = ExposureBuffer.next_frame) equal
    the oracle's host-side blend bit for bit; then statistics, range and RGBA8 of the result."""
    import torch
    spec = scenes.small_random(7)
    W, H = 96, 64
    cams = [scenes.make_camera(W, H, init_h=a) for a in (0.5, 0.6, 0.7)]
    w, root = oracle.build_scene(spec)
    ref = np.zeros(W * H * 3, np.float32)
    ctx = rtamd.Context(0)
    try:
        ctx.upload(rtamd.build_scene(spec))
        buf = torch.full((H, W, 3), 123.0, dtype=torch.float32, device="cuda")
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        for k, cam in enumerate(cams):
            cfg = scenes.make_config(3, col_weight=1 / (1 + k))
            w.trace_frame(root, cam, cfg, rgb=ref, nthreads=4)
            ctx.trace_rows_device(cam, cfg, 0, 1, 8, buf.data_ptr(), s.cuda_stream)
        s.synchronize()
        got = buf.reshape(-1).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        st = ctx.exposure_stats_device(buf.data_ptr(), W * H, s.cuda_stream)
        ref_st = oracle.exposure_stats(ref)
        _stats_close([st.mean, st.variance, st.absdev], ref_st, W * H)
        lo, hi = oracle.tonemap_range(1, ref_st)
        out = torch.zeros(4 * W * H, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()                    # the fill runs on torch's stream, the kernel on `s`
        ctx.tonemap_device(buf.data_ptr(), W * H, lo, hi, out.data_ptr(), s.cuda_stream)
        s.synchronize()
        assert np.array_equal(out.cpu().numpy(), oracle.tonemap(ref, lo, hi))
    finally:
        ctx.close()
        w.close()


@pytest.mark.gpu
def test_stats_full_hd_frame():
    """1080p config-1-scene frame: statistics within n * 2^-52 (relative), RGBA8 bit-exact."""
    import torch
    spec = scenes.config1_spheres()
    W, H = 1920, 1080
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(2)
    ctx = rtamd.Context(0)
    try:
        ctx.upload(rtamd.build_scene(spec))
        buf = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        ctx.trace_rows_device(cam, cfg, 0, 1, 8, buf.data_ptr(), s.cuda_stream)
        st = ctx.exposure_stats_device(buf.data_ptr(), W * H, s.cuda_stream)
        host = buf.reshape(-1).cpu().numpy()
        ref_st = oracle.exposure_stats(host)
        _stats_close([st.mean, st.variance, st.absdev], ref_st, W * H)
        lo, hi = oracle.tonemap_range(1, ref_st)
        out = torch.zeros(4 * W * H, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        ctx.tonemap_device(buf.data_ptr(), W * H, lo, hi, out.data_ptr(), s.cuda_stream)
        s.synchronize()
        assert np.array_equal(out.cpu().numpy(), oracle.tonemap(host, lo, hi))
    finally:
        ctx.close()
