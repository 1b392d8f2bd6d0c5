"""The C-ABI library loads, exports every symbol include/rt.h declares, and its struct layouts
match the ctypes mirror.  No compute calls (these run without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import rtamd
from rtamd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w[\w\s\*]*?\b(rt_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_symbols():
    assert _declared() == sorted(abi.EXPORTS)


def test_library_exports_every_symbol():
    lib = rtamd.load_library()
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", rtamd.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (rt_\w+)$", out, re.M))
    assert set(_declared()) <= exported
    assert lib.rt_abi_version() == 5


def test_struct_layouts_match_header(tmp_path):
    prog = tmp_path / "sz.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "rt.h"\nint main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n",'
                    'sizeof(rt_shade),sizeof(rt_scene_desc),sizeof(rt_camera_desc),sizeof(rt_config_desc),'
                    'sizeof(rt_stats),sizeof(rt_create_desc),sizeof(rt_entity_in),offsetof(rt_scene_desc,substance_ri),'
                    'sizeof(rt_exposure_stats),sizeof(rt_image_desc),offsetof(rt_scene_desc,images),'
                    'sizeof(rt_update_stats),offsetof(rt_config_desc,sky_image),sizeof(rt_ctx_info),'
                    'offsetof(rt_create_desc,devices));'
                    'printf("%zu %zu %zu\\n",sizeof(rt_edit_desc),offsetof(rt_edit_desc,scatter),'
                    'offsetof(rt_edit_desc,substance_ri));'
                    'printf("%zu %zu %d\\n",sizeof(rt_light),offsetof(rt_light,rgb),RT_MAX_LIGHTS);return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [C.sizeof(abi.rt_shade), C.sizeof(abi.rt_scene_desc), C.sizeof(abi.rt_camera_desc),
            C.sizeof(abi.rt_config_desc), C.sizeof(abi.rt_stats), C.sizeof(abi.rt_create_desc),
            C.sizeof(abi.rt_entity_in), abi.rt_scene_desc.substance_ri.offset, C.sizeof(abi.rt_exposure_stats),
            C.sizeof(abi.rt_image_desc), abi.rt_scene_desc.images.offset, C.sizeof(abi.rt_update_stats),
            abi.rt_config_desc.sky_image.offset, C.sizeof(abi.rt_ctx_info), abi.rt_create_desc.devices.offset,
            C.sizeof(abi.rt_edit_desc), abi.rt_edit_desc.scatter.offset, abi.rt_edit_desc.substance_ri.offset,
            C.sizeof(abi.rt_light), abi.rt_light.rgb.offset, abi.RT_MAX_LIGHTS]
    assert got == want


def test_null_arguments_are_rejected_without_gpu():
    lib = rtamd.load_library()
    assert lib.rt_create(None, None) == abi.RT_E_INVALID
    assert b"null" in lib.rt_last_error()
    assert lib.rt_upload_scene(None, None) == abi.RT_E_INVALID
    assert lib.rt_trace_frame(None, None, None, None, None, None, None, None) == abi.RT_E_INVALID
    assert lib.rt_exposure_stats_device(None, None, 0, None, None) == abi.RT_E_INVALID
    assert lib.rt_tonemap_device(None, None, 1, 0.0, 1.0, None, None) == abi.RT_E_INVALID
    assert lib.rt_trace_frame_device(None, None, None, None, None) == abi.RT_E_INVALID
    assert lib.rt_frame_fault(None, None) == abi.RT_E_INVALID
    assert lib.rt_ctx_info_get(None, None) == abi.RT_E_INVALID
    assert lib.rt_set_lights(None, None, 0, 0.0) == abi.RT_E_INVALID


def test_create_rejects_bad_device_lists_without_gpu():
    """Without a GPU rt_create reports RT_E_NODEVICE before it looks at the list; the list checks
    themselves (count 0..8, ordinals, stripe) run first on a GPU host (tests/test_multi_device.py)."""
    lib = rtamd.load_library()
    cd = abi.rt_create_desc(n_devices=9)
    h = C.c_void_p()
    assert lib.rt_create(C.byref(cd), C.byref(h)) in (abi.RT_E_INVALID, abi.RT_E_NODEVICE)
    assert not h.value


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(RuntimeError, match="not found"):
        rtamd.load_library(str(tmp_path / "nope.so"))
