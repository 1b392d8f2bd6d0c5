"""Multi-device contexts (include/rt.h rt_create_desc.devices) on a real MI355X.

One context splits each frame into row stripes dealt round-robin over its devices, traces every
part on its device, gathers the parts on devices[0] (RCCL ncclGather, or device copies) and
de-interleaves them.  The test box has one GPU, so the split runs as several parts on that GPU
(the device-copy gather; RCCL admits one rank per GPU) and the RCCL path as a one-rank
communicator (RT_GATHER=rccl).  Results must equal the single-device frame and the oracle bit for
bit: the partition changes scheduling only.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
import rtamd
from rtamd import abi, scenes

pytestmark = pytest.mark.gpu

KEYS = ("rgb", "hit_entity", "hit_node", "status")


def _same(a, b):
    for k in KEYS:
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k


def _ctx(spec_scene, **kw):
    c = rtamd.Context(**kw)
    c.upload(spec_scene)
    return c


@pytest.fixture(scope="module")
def small3():
    spec = scenes.small_random(3)
    return spec, rtamd.build_scene(spec)


@pytest.fixture(scope="module")
def single(small3):
    c = _ctx(small3[1], device=0)
    yield c
    c.close()


@pytest.mark.parametrize("devices,stripe", [([0, 0], 8), ([0, 0, 0], 1), ([0] * 8, 8), ([0] * 5, 13), ([0, 0], 500)])
def test_parts_on_one_gpu_equal_single_device_and_oracle(small3, single, devices, stripe):
    """n parts of the frame on one GPU through the multi-device code path: stripes of 1, 8, 13 and
    500 rows (a partial last stripe; more rows than the frame), 2-8 parts."""
    spec, scene = small3
    cam, cfg = scenes.make_camera(160, 120), scenes.make_config(3)
    ref = single.trace_frame(cam, cfg, allow_fault=True)
    m = _ctx(scene, devices=devices, stripe_rows=stripe)
    try:
        info = m.info()
        assert info["n_devices"] == len(devices) and info["stripe_rows"] == stripe and info["gather"] == "peer"
        got = m.trace_frame(cam, cfg, allow_fault=True)
        _same(ref, got)
        assert got["rc"] == ref["rc"]
        assert got["stats"].counters() == ref["stats"].counters()       # summed over the parts
        _same(ref, m.trace_frame(cam, cfg, stats=False, allow_fault=True))
    finally:
        m.close()
    w, root = oracle.build_scene(spec)
    r = w.trace_frame(root, cam, cfg, nthreads=8)
    assert np.array_equal(r["rgb"].view(np.uint32), got["rgb"].view(np.uint32))
    assert np.array_equal(r["hit_entity"], got["hit_entity"]) and np.array_equal(r["hit_node"], got["hit_node"])


def test_rccl_gather_one_rank(small3, single, monkeypatch):
    """The RCCL path (ncclCommInitAll, ncclGather per output array, ncclScatter for a blend, the
    de-interleave kernel) with a one-rank communicator: the frame equals the single-device one."""
    spec, scene = small3
    cam, cfg = scenes.make_camera(160, 120), scenes.make_config(3)
    monkeypatch.setenv("RT_GATHER", "rccl")
    m = _ctx(scene, devices=[0])
    try:
        assert m.info()["gather"] == "rccl"
        _same(single.trace_frame(cam, cfg, allow_fault=True), m.trace_frame(cam, cfg, allow_fault=True))
        bcfg = scenes.make_config(3, col_weight=0.25)
        old = np.random.default_rng(1).uniform(0, 2, 160 * 120 * 3).astype(np.float32)
        a = single.trace_frame(cam, bcfg, rgb=old.copy(), allow_fault=True)
        b = m.trace_frame(cam, bcfg, rgb=old.copy(), allow_fault=True)
        _same(a, b)
    finally:
        m.close()


@pytest.mark.parametrize("stats", [True, False])
@pytest.mark.parametrize("devices", [[0, 0, 0], [0, 0, 0, 0, 0, 0, 0]])
def test_blend_over_parts(small3, single, devices, stats):
    """ExposureBuffer blend (col_weight != 1) on a split frame: the current frame is dealt out to
    the parts first (the gather path: k_stripes + scatter; without counters: each part's stripes
    copied from the host buffer to its device), each part blends in binary64 as the one-device frame
    does."""
    spec, scene = small3
    cam, cfg = scenes.make_camera(64, 45), scenes.make_config(2, col_weight=1 / 3)
    old = np.random.default_rng(0).uniform(0, 2, 64 * 45 * 3).astype(np.float32)
    m = _ctx(scene, devices=devices)
    try:
        _same(single.trace_frame(cam, cfg, rgb=old.copy(), allow_fault=True),
              m.trace_frame(cam, cfg, rgb=old.copy(), stats=stats, allow_fault=True))
    finally:
        m.close()
    w, root = oracle.build_scene(spec)
    ref = w.trace_frame(root, cam, cfg, rgb=old.copy())
    got = single.trace_frame(cam, cfg, rgb=old.copy(), allow_fault=True)
    assert np.array_equal(ref["rgb"].view(np.uint32), got["rgb"].view(np.uint32))


@pytest.mark.parametrize("direct", ["1", "0"])
@pytest.mark.parametrize("ids", [True, False])
@pytest.mark.parametrize("devices,stripe,wh", [([0, 0], 8, (160, 120)), ([0] * 8, 8, (200, 135)),
                                               ([0] * 3, 5, (101, 37)), ([0] * 5, 500, (64, 48))])
def test_host_frame_parts_copied_per_device(small3, single, devices, stripe, wh, ids, direct, monkeypatch):
    """The multi-device host frame without counters: each device copies its own stripes into the host
    buffer (2D copies; a partial last stripe; empty parts), ids on and off; RT_HOST_DIRECT=0 is the
    gather to devices[0] and one D2H.  Both equal the one-device frame bit for bit."""
    monkeypatch.setenv("RT_HOST_DIRECT", direct)
    spec, scene = small3
    cam, cfg = scenes.make_camera(*wh), scenes.make_config(3)
    ref = single.trace_frame(cam, cfg, stats=False, allow_fault=True)
    m = _ctx(scene, devices=devices, stripe_rows=stripe)
    try:
        for _ in range(2):
            got = m.trace_frame(cam, cfg, ids=ids, stats=False, allow_fault=True)
            assert got["rc"] == ref["rc"]
            assert np.array_equal(ref["rgb"].view(np.uint32), got["rgb"].view(np.uint32))
            if ids:
                _same(ref, got)
    finally:
        m.close()


@pytest.mark.parametrize("gather", ["peer", "rccl"])
def test_trace_frame_device(small3, single, gather, monkeypatch):
    """rt_trace_frame_device into a torch tensor on cuda:0, ordered on a torch stream: equals the
    host-buffer frame; several frames back to back (buffers reused in stream order); blends."""
    import torch
    spec, scene = small3
    W, H = 200, 150
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(3)
    monkeypatch.setenv("RT_GATHER", gather)
    m = _ctx(scene, devices=[0, 0, 0] if gather == "peer" else [0])
    try:
        assert m.info()["gather"] == gather
        ref = single.trace_frame(cam, cfg, allow_fault=True)["rgb"]
        out = torch.full((H, W, 3), float("nan"), dtype=torch.float32, device="cuda:0")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                m.trace_frame_device(cam, cfg, out.data_ptr(), s.cuda_stream)
            got = out.cpu().numpy().reshape(-1)              # ordered after the frame by the stream
        assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))
        bcfg = scenes.make_config(3, col_weight=0.5)
        with torch.cuda.stream(s):
            m.trace_frame_device(cam, bcfg, out.data_ptr(), s.cuda_stream)
            blended = out.cpu().numpy().reshape(-1)
        want = single.trace_frame(cam, bcfg, rgb=got.copy(), allow_fault=True)["rgb"]
        assert np.array_equal(want.view(np.uint32), blended.view(np.uint32))
    finally:
        m.close()


def _throwing_scene():
    """Config 1's spheres, all TRANSMISSION with GLASS, seen from an undefined substance (room box and
    default substance undefined): the first refraction reads undefined.refractive_index, where the
    reference throws (src/raytracer.ts:135-150, 238-249)."""
    spec = scenes.config1_spheres()
    e, sh = spec.entities.copy(), spec.shades.copy()
    sh["response"][:] = abi.RT_RESP_TRANSMISSION
    sh["light"][:] = 0
    e["substance"][:] = 2
    e["substance"][-1] = -1
    return scenes.SceneSpec("throws", e, sh)


def test_frame_fault_reports_reference_throws():
    """The host path returns RT_E_FAULT, the device paths report it through rt_frame_fault, and a
    clean frame clears it (the flag is reset per frame)."""
    import torch
    bad = rtamd.build_scene(_throwing_scene())
    good = rtamd.build_scene(scenes.small_random(3))
    cam, cfg = scenes.make_camera(128, 128), scenes.make_config(5, default_substance=-1)
    out = torch.zeros((128, 128, 3), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    for kw in (dict(device=0), dict(devices=[0, 0])):
        m = _ctx(bad, **kw)
        try:
            r = m.trace_frame(cam, cfg, allow_fault=True)
            assert r["rc"] == abi.RT_E_FAULT and (r["status"] == 2).any()
            m.trace_frame_device(cam, cfg, out.data_ptr())
            assert m.frame_fault()
            if "device" in kw:
                m.trace_rows_device(cam, cfg, 0, 1, 8, out.data_ptr())
                assert m.frame_fault()
            m.upload(good)
            assert m.trace_frame(cam, cfg)["rc"] == 0
            m.trace_frame_device(cam, cfg, out.data_ptr())
            assert not m.frame_fault()
            if "device" in kw:
                m.trace_rows_device(cam, cfg, 0, 1, 8, out.data_ptr())
                assert not m.frame_fault()
        finally:
            m.close()


@pytest.mark.parametrize("stats", [True, False])
@pytest.mark.parametrize("kw", [dict(device=0), dict(devices=[0, 0, 0], stripe_rows=3)])
def test_throw_keeps_the_reference_partial_frame(kw, stats):
    """After a throw the reference's ExposureBuffer holds the pixels traced before the first throwing
    pixel in scan order; that pixel and all later ones keep their previous value
    (src/raytracer.ts:318-329).  rt_trace_frame leaves the same buffer, bit for bit with the oracle."""
    spec = _throwing_scene()
    cam, cfg = scenes.make_camera(96, 72), scenes.make_config(5, default_substance=-1, col_weight=0.5)
    old = np.random.default_rng(5).random(96 * 72 * 3, dtype=np.float32)
    w, root = oracle.build_scene(spec)
    try:
        want = w.trace_frame(root, cam, cfg, rgb=old.copy(), abort=True)
    finally:
        w.close()
    st = want["status"]
    assert (st == 2).any() and (st == 0).any()
    m = _ctx(rtamd.build_scene(spec), **kw)
    try:
        got = m.trace_frame(cam, cfg, rgb=old.copy(), stats=stats, allow_fault=True)
    finally:
        m.close()
    assert got["rc"] == abi.RT_E_FAULT
    assert np.array_equal(got["status"], st)
    assert np.array_equal(got["rgb"].view(np.uint32), want["rgb"].view(np.uint32))
    idx = oracle.scan_index(96, 72)
    kept = idx >= idx[st.ravel() >= 2].min()
    assert kept.any() and (~kept).any()
    assert np.array_equal(got["rgb"].reshape(-1, 3)[kept], old.reshape(-1, 3)[kept])


@pytest.mark.parametrize("parts", [4, 8])
def test_config3_split_over_parts(parts):
    """BASELINE config 3 at 1920x1080 as 4 and 8 parts (the driver's N = 8 workload, one GPU's share
    each): bit-identical to the one-part frame, which test_baseline_config_full_frame holds to the
    oracle."""
    factory, W, H, refmax = scenes.WORKLOADS["config3"]
    scene = rtamd.build_scene(factory())
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(refmax)
    a = _ctx(scene, device=0)
    b = _ctx(scene, devices=[0] * parts)
    try:
        _same(a.trace_frame(cam, cfg, stats=False), b.trace_frame(cam, cfg, stats=False))
    finally:
        a.close()
        b.close()


def test_bad_device_lists():
    L = rtamd.load_library()
    h = C.c_void_p()
    cd = abi.rt_create_desc(n_devices=9)
    assert L.rt_create(C.byref(cd), C.byref(h)) == abi.RT_E_INVALID and not h.value
    cd = abi.rt_create_desc(n_devices=2)
    cd.devices[0], cd.devices[1] = 0, 4096
    assert L.rt_create(C.byref(cd), C.byref(h)) == abi.RT_E_NODEVICE and not h.value
    cd = abi.rt_create_desc(n_devices=1, stripe_rows=-1)
    assert L.rt_create(C.byref(cd), C.byref(h)) == abi.RT_E_INVALID and not h.value
    m = rtamd.Context(devices=[0, 0])
    try:
        with pytest.raises(rtamd.RtError):               # the per-rank entry point is single-device
            m.upload(rtamd.build_scene(scenes.config1_spheres()))
            m.trace_rows_device(scenes.make_camera(8, 8), scenes.make_config(1), 0, 1, 8, 0)
    finally:
        m.close()


def test_device_restored_after_calls():
    """Entry points leave the caller's current device as they found it (torch keeps its own)."""
    import torch
    torch.cuda.set_device(0)
    m = rtamd.Context(devices=[0, 0])
    try:
        m.upload(rtamd.build_scene(scenes.config1_spheres()))
        m.trace_frame(scenes.make_camera(32, 32), scenes.make_config(2))
        assert torch.cuda.current_device() == 0
    finally:
        m.close()


def _n_gpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif("_n_gpus() < 2", reason="needs two distinct GPUs (the parity box has one)")
@pytest.mark.parametrize("gather", ["peer", "rccl"])
def test_distinct_gpus_equal_single_device(small3, single, gather, monkeypatch):
    """devices=[0, 1]: the distinct-GPU path (peer access or a two-rank RCCL communicator, cross-device
    event ordering) gives the one-device frame, the blend and the reference's partial frame after a
    throw.  Runs only where hipGetDeviceCount() >= 2; the one-GPU box skips it (README)."""
    spec, scene = small3
    monkeypatch.setenv("RT_GATHER", gather)
    cam, cfg = scenes.make_camera(160, 120), scenes.make_config(3)
    m = _ctx(scene, devices=[0, 1], stripe_rows=8)
    try:
        assert m.info()["gather"] == gather and m.info()["n_devices"] == 2
        _same(single.trace_frame(cam, cfg, allow_fault=True), m.trace_frame(cam, cfg, allow_fault=True))
        bcfg = scenes.make_config(3, col_weight=0.25)
        old = np.random.default_rng(2).uniform(0, 2, 160 * 120 * 3).astype(np.float32)
        _same(single.trace_frame(cam, bcfg, rgb=old.copy(), allow_fault=True),
              m.trace_frame(cam, bcfg, rgb=old.copy(), allow_fault=True))
    finally:
        m.close()
    tspec = _throwing_scene()
    tcam, tcfg = scenes.make_camera(96, 72), scenes.make_config(5, default_substance=-1, col_weight=0.5)
    old = np.random.default_rng(5).random(96 * 72 * 3, dtype=np.float32)
    tscene = rtamd.build_scene(tspec)
    a, b = _ctx(tscene, device=0), _ctx(tscene, devices=[0, 1], stripe_rows=3)
    try:
        ra = a.trace_frame(tcam, tcfg, rgb=old.copy(), allow_fault=True)
        rb = b.trace_frame(tcam, tcfg, rgb=old.copy(), allow_fault=True)
        assert ra["rc"] == rb["rc"] == abi.RT_E_FAULT
        _same(ra, rb)
    finally:
        a.close()
        b.close()
