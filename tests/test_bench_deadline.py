"""bench.py's wall-time bound, on CPU: the JSON line is printed before the deadline even when every
optional phase after the timed frames hangs.

A fake `rocprofv3` and a fake `node` that sleep forever go first on PATH; report() (the part of
bench.py that runs after the timed GPU frames) is fed a synthetic timed-frames result of the config-1
scene.  The rocprofv3 passes and the JS runs must be killed at their limits, the CPU baseline must
fall back to the C oracle, and the record must carry the notes.  A second case hangs a phase inside
the process itself: the watchdog must print the record and exit."""
import json
import os
import stat
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = textwrap.dedent('''
    import sys, time, types
    sys.path.insert(0, %(root)r)
    import bench
    from rtamd import scenes
    import rtamd
    mode, deadline_s = sys.argv[1], float(sys.argv[2])
    factory, W, H, refmax = scenes.WORKLOADS["config1"]
    spec = factory()
    scene = rtamd.build_scene(spec)
    tot = dict(segments=73728, n_ret=1, n_slot=1, n_loc=1, n_sph=1, n_box=1, n_tri=1, n_hit=1, primary=65536,
               n_warn=0, n_fault=0, n_cull=1, n_exact=1)
    res = dict(tot=tot, elapsed=0.01, elapsed_serial=0.02, elapsed_moving=0.011, warmup_frames=16, kernel_ms=0.1, same=True, host=None,
               exposure=None, P=16, mode="one GPU", collective=None, n_gpus=1)
    args = types.SimpleNamespace(steps=32, warmup=3, config="config1", stripe=8, cpu_budget=2.0, no_profile=False,
                                 profile_out=None, no_js=False, deadline=deadline_s)
    deadline = bench.Deadline(deadline_s, t0=time.monotonic())
    rep = bench.Reporter()
    rep.arm(deadline, grace_s=2.0)
    if mode == "hang":
        def forever(*a, **k):
            time.sleep(10000)
        bench.cpu_baseline = forever
    bench.report(args, res, spec, scene, W, H, refmax, 0.0, deadline, rep)
''')


def _fake_bin(tmp_path):
    d = tmp_path / "bin"
    d.mkdir()
    for name in ("rocprofv3", "node"):
        p = d / name
        # ignores SIGTERM, and leaves a grandchild holding stdout: only a process-group kill ends it
        p.write_text("#!/bin/bash\ntrap '' TERM\nsleep 100000 &\nwait\n")
        p.chmod(p.stat().st_mode | stat.S_IEXEC)
    return str(d)


def _run(tmp_path, mode, deadline_s):
    drv = tmp_path / "drv.py"
    drv.write_text(DRIVER % dict(root=ROOT))
    env = dict(os.environ, PATH=_fake_bin(tmp_path) + os.pathsep + os.environ["PATH"])
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(drv), mode, str(deadline_s)], env=env, capture_output=True, text=True,
                       timeout=deadline_s + 120)
    wall = time.monotonic() - t0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, wall, lines


def test_json_line_before_deadline_with_hanging_profiler_and_node(tmp_path):
    deadline_s = 45.0
    r, wall, lines = _run(tmp_path, "normal", deadline_s)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    # the run's own clock: imports of the child are outside the Deadline here, so bound the phases
    assert rec["wall"]["emitted_s"] < 400
    assert wall < deadline_s + 60, wall
    notes = rec["roofline"]["profile_notes"]
    assert any("killed at its" in n or "skipped" in n for n in notes), notes
    assert rec["value"] > 0 and rec["roofline"]["frac"] is None
    cpu = rec["cpu_baseline"]
    assert cpu is not None and "js_error" in cpu and cpu["kind"] == "port"     # C oracle took over
    assert rec["js_frame"]["error"]


def test_watchdog_prints_record_when_a_phase_hangs(tmp_path):
    deadline_s = 20.0
    r, wall, lines = _run(tmp_path, "hang", deadline_s)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert any("watchdog" in s for s in rec["skipped_phases"]), rec.get("skipped_phases")
    assert rec["cpu_baseline"] is None
    assert wall < deadline_s + 60, wall
