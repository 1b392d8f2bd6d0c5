"""The RCCL call sequence of multi-device frames, checked on a CPU against a recording stub.

frame_multi (raytracer.js_amd/csrc/rt_api.hip) issues its collectives through rt_rccl_frame
(rt_internal.h); rt_debug_rccl_frames drives that same function over placeholder streams and
buffers for `frames` frames on `n_ctx` contexts (frames in flight, each context with its own
communicators over the same devices), loading librccl's entry points from RT_RCCL_LIB, which points
at tests/stub_rccl.c built here.  The stub records every call in order.  Checked:

* one gather group per frame, and one scatter group before it for a blend, each holding only that
  frame's context's communicators, one call per device per array;
* every device sees the same sequence of (context, operation, array) calls — the order that keeps
  concurrent communicators on the same GPUs from deadlocking;
* roots (device 0), element counts and datatypes; each device's send buffer is its own part, the
  receive buffer device 0's stack at the layout the de-interleave kernel reads;
* a blend's scatter comes before every device's trace of that frame, the gather after all of them;
* communicators: one ncclCommInitAll of all devices per context, all destroyed at the end.

What this does not check: that RCCL itself, or the GPUs, execute the calls (no multi-GPU box is
available to this build; DESIGN.md §7 states that).
"""
import ctypes as C
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "raytracer.js_amd", "lib", "librt_amd.so")
OP_INIT, OP_DESTROY, OP_GS, OP_GE, OP_GATHER, OP_SCATTER, OP_MARK = range(1, 8)
F32, I32, U8 = 7, 2, 1

CHILD = r"""
import ctypes as C, json, sys
sys.path.insert(0, %(py)r)
from rtamd import abi
lib = abi.declare(C.CDLL(%(lib)r))
stub = C.CDLL(%(stub)r)
class Rec(C.Structure):
    _fields_ = [("op", C.c_int32), ("init", C.c_int32), ("rank", C.c_int32), ("dtype", C.c_int32),
                ("root", C.c_int32), ("pad", C.c_int32), ("send", C.c_uint64), ("recv", C.c_uint64),
                ("count", C.c_uint64), ("stream", C.c_uint64)]
stub.stub_mark.argtypes = [C.c_int32, C.c_int32]
stub.stub_get.argtypes = [C.c_int, C.POINTER(Rec)]
hook = abi.TRACE_HOOK(lambda x, k: stub.stub_mark(x, k))
rc = lib.rt_debug_rccl_frames(*%(args)r, hook)
out = []
r = Rec()
for i in range(stub.stub_count()):
    stub.stub_get(i, C.byref(r))
    out.append([r.op, r.init, r.rank, r.dtype, r.root, r.send, r.recv, r.count, r.stream])
print(json.dumps({"rc": rc, "err": lib.rt_last_error().decode(), "log": out}))
"""


@pytest.fixture(scope="module")
def stub(tmp_path_factory):
    if not os.path.exists(LIB):
        pytest.fail("librt_amd.so not built (run __graft_entry__.build())")
    so = str(tmp_path_factory.mktemp("stub") / "libstub_rccl.so")
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", os.path.join(ROOT, "tests", "stub_rccl.c"), "-o", so], check=True)
    return so


def _run(stub, n_dev, n_ctx, frames, W, H, stripe, blend, ids):
    src = CHILD % dict(py=os.path.join(ROOT, "raytracer.js_amd", "python"), lib=LIB, stub=stub,
                       args=[n_dev, n_ctx, frames, W, H, stripe, int(blend), int(ids)])
    env = dict(os.environ, RT_RCCL_LIB=stub)
    p = subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["rc"] == 0, res["err"]
    return res["log"]


def _part_rows(H, part, n, stripe):
    rows = 0
    for s in range(part, (H + stripe - 1) // stripe, n):
        rows += min(stripe, H - s * stripe)
    return rows


def _check(log, n_dev, n_ctx, frames, W, H, stripe, blend, ids):
    PS = max(_part_rows(H, p, n_dev, stripe) for p in range(n_dev)) * W
    # communicators: one InitAll of n_dev ranks per context, in context order, devices 0..n-1
    inits = [e for e in log if e[0] == OP_INIT]
    assert [(e[1], e[2], e[4], e[7]) for e in inits] == [(x, k, k, n_dev) for x in range(n_ctx) for k in range(n_dev)]
    assert log[:len(inits)] == inits
    destroys = [(e[1], e[2]) for e in log if e[0] == OP_DESTROY]
    assert sorted(destroys) == [(x, k) for x in range(n_ctx) for k in range(n_dev)]
    body = [e for e in log if e[0] not in (OP_INIT, OP_DESTROY)]
    arrays = [(F32, 3 * PS, 12)] + ([(I32, PS, 4), (I32, PS, 4), (U8, PS, 1)] if ids else [])
    i = 0
    for f in range(frames):
        x = f % n_ctx
        cx = x + 1
        base = cx << 40 | 0xFF << 32
        stack_off = [0, n_dev * PS * 12, n_dev * PS * 16, n_dev * PS * 20]
        stream = [cx << 24 | (k + 1) << 8 for k in range(n_dev)]
        part = lambda k, a: cx << 40 | (k + 1) << 32 | (a + 1) << 24   # noqa: E731
        if blend:
            # the scatter group: device 0's dealt frame to every part, before any trace of the frame
            assert body[i][0] == OP_GS, (f, body[i])
            grp = body[i + 1:i + 1 + n_dev]
            assert body[i + 1 + n_dev][0] == OP_GE
            for k, e in enumerate(grp):
                op, init, rank, dt, root, send, recv, count, st = e
                assert (op, init, rank, dt, root) == (OP_SCATTER, x, k, F32, 0), e
                assert (send, recv, count, st) == (base, part(k, 0), 3 * PS, stream[k]), e
            i += n_dev + 2
        # every device's trace of this frame, on this context
        marks = body[i:i + n_dev]
        assert [(e[0], e[1], e[2]) for e in marks] == [(OP_MARK, x, k) for k in range(n_dev)], (f, marks)
        i += n_dev
        # one gather group: array-major, devices in order, only this context's communicators
        assert body[i][0] == OP_GS, (f, body[i])
        n_call = len(arrays) * n_dev
        grp = body[i + 1:i + 1 + n_call]
        assert body[i + 1 + n_call][0] == OP_GE, (f, body[i + 1 + n_call])
        for j, e in enumerate(grp):
            a, k = divmod(j, n_dev)
            dt, count, _ = arrays[a]
            op, init, rank, edt, root, send, recv, ecount, st = e
            assert (op, init, rank, edt, root) == (OP_GATHER, x, k, dt, 0), e
            assert (send, recv, ecount, st) == (part(k, a), base + stack_off[a], count, stream[k]), e
        i += n_call + 2
    assert i == len(body)
    # the same (context, op, array) sequence on every device: what each device's communicators see
    per_dev = {k: [] for k in range(n_dev)}
    for e in body:
        if e[0] in (OP_GATHER, OP_SCATTER):
            per_dev[e[2]].append((e[1], e[0], e[3], e[7]))
    for k in range(1, n_dev):
        assert per_dev[k] == per_dev[0], k
    # groups per frame: 1 (+1 for a blend)
    assert sum(e[0] == OP_GS for e in body) == frames * (2 if blend else 1)


@pytest.mark.parametrize("blend,ids", [(False, False), (True, False), (False, True), (True, True)])
def test_eight_devices_four_contexts(stub, blend, ids):
    """N = 8 devices, P = 4 frames in flight (bench.py's multi-device layout), 3840x2160 (config 4)."""
    args = (8, 4, 10, 3840, 2160, 8, blend, ids)
    _check(_run(stub, *args), *args)


@pytest.mark.parametrize("n_dev,n_ctx,H,stripe", [(2, 1, 1080, 8), (3, 2, 37, 5), (5, 3, 13, 500), (8, 16, 1080, 8)])
def test_other_device_and_context_counts(stub, n_dev, n_ctx, H, stripe):
    """Ragged parts (rows not a multiple of N stripes, empty parts) and up to 16 frames in flight."""
    for blend in (False, True):
        args = (n_dev, n_ctx, 2 * n_ctx + 1, 101, H, stripe, blend, True)
        _check(_run(stub, *args), *args)


def test_bad_arguments_are_rejected(stub):
    sys.path.insert(0, os.path.join(ROOT, "raytracer.js_amd", "python"))
    from rtamd import abi
    lib = abi.declare(C.CDLL(LIB))
    hook = abi.TRACE_HOOK(lambda x, k: None)
    assert lib.rt_debug_rccl_frames(0, 1, 1, 8, 8, 8, 0, 0, hook) == abi.RT_E_INVALID
    assert lib.rt_debug_rccl_frames(9, 1, 1, 8, 8, 8, 0, 0, hook) == abi.RT_E_INVALID
    assert lib.rt_debug_rccl_frames(2, 1, 1, 8, 8, 0, 0, 0, hook) == abi.RT_E_INVALID
