"""The JS drop-in's trace_frame() wall time (node -> N-API -> librt_amd.so, ExposureBuffer.pixels
filled): a BASELINE config's scene dumped to JSON, built as reference-shaped objects by
tests/js/run_dropin.js, then N frames timed without and with options.stats (work counters).

python tools/js_frame_time.py [--config config3] [--frames 10]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracer.js_amd", "python"), ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from rtamd import scenes  # noqa: E402
from test_js_dropin import RUNNER, _dump  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--frames", type=int, default=10)
    a = ap.parse_args()
    factory, W, H, refmax = scenes.WORKLOADS[a.config]
    with tempfile.TemporaryDirectory() as td:
        path = _dump(Path(td), factory(), scenes.make_camera(W, H), scenes.make_config(refmax))
        r = subprocess.run(["node", "--max-old-space-size=16384", RUNNER, path, os.path.join(td, "out"),
                            "--repeat", str(a.frames)], capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            sys.exit(r.stdout[-2000:] + r.stderr[-2000:])
        rep = json.loads(Path(td, "out.repeat.json").read_text())
    med = {k: float(np.median(v)) for k, v in rep.items()}
    print(json.dumps(dict(config=a.config, frames=a.frames, js_trace_frame_ms_median=round(med["frame_ms"], 3),
                          js_trace_frame_ms_median_with_stats=round(med["frame_ms_stats"], 3), raw=rep)))


if __name__ == "__main__":
    main()
