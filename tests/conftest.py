"""Shared test setup: marker registration and import paths.

`-m "not gpu"` runs the oracle-vs-reference-KAT checks, host logic and ABI load checks on CPU;
`-m gpu` runs the HIP parity tests through the C ABI on a real MI355X.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Frames of up to RT_FUSE_MAX pixels (default 2^18) of light scenes run the fused one-kernel trace.
# Most parity tests render small frames; they set the threshold to 0 so that they exercise the split
# walk / first-hit / shade passes that every large frame runs.  Tests of the small-frame default
# (test_small_frames_fused_default_equals_oracle) create their contexts with it restored.
os.environ.setdefault("RT_FUSE_MAX", "0")
for p in (ROOT, os.path.join(ROOT, "raytracer.js_amd", "python"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        return json.load(f)
