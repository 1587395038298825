"""The C-ABI library: it loads, exports every function include/*.h declares,
and fails loudly (no CPU fallback) where no HIP device is usable.  CPU-only:
no compute call is made here."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import PKG, ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in ("rtc.h", "rtc_scene.h")]
LIB = os.path.join(PKG, "rtc_amd", "_lib", "librtc.so")
RT_ERR_INVALID, RT_ERR_NO_DEVICE = -1, -3


def declared_functions():
    names = []
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*(rt_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_headers_declare_the_boundary():
    names = declared_functions()
    for must in ("rt_context_create", "rt_scene_upload", "rt_render", "rt_render_device", "rt_color_at",
                 "rt_scene_load_yaml", "rt_camera_make", "rt_assemble_shards"):
        assert must in names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rt_\w+)$", out, flags=re.M))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, f"declared but not exported: {missing}"


def test_python_mirror_lists_every_symbol(rtc):
    assert sorted(rtc.EXPORTED_SYMBOLS) == declared_functions()


def test_abi_version_and_last_error(rtc):
    assert rtc.abi_version() == rtc.RT_ABI_VERSION == 3
    lib = C.CDLL(LIB)
    lib.rt_last_error.restype = C.c_char_p
    assert lib.rt_last_error() is not None


def test_null_arguments_are_rejected():
    lib = C.CDLL(LIB)
    assert lib.rt_device_count(None) == RT_ERR_INVALID
    assert lib.rt_context_create(0, None) == RT_ERR_INVALID
    assert lib.rt_shard_rows(1080, 0, None) == RT_ERR_INVALID
    assert lib.rt_shard_row_map(1080, 0, None, None) == RT_ERR_INVALID
    assert lib.rt_context_create_multi(None, 1, None) == RT_ERR_INVALID
    assert lib.rt_comm_unique_id(None) == RT_ERR_INVALID
    assert lib.rt_context_create_rank(0, 2, 5, None, None) == RT_ERR_INVALID


def test_no_device_means_no_multi_gpu_context(rtc):
    if rtc.device_count() > 0:
        pytest.skip("a HIP device is visible here")
    with pytest.raises(rtc.RenderError) as e:
        rtc.Context.multi([0])
    assert e.value.code == RT_ERR_NO_DEVICE


def test_no_device_means_an_error_not_a_fallback(rtc):
    if rtc.device_count() > 0:
        pytest.skip("a HIP device is visible here")
    with pytest.raises(rtc.RenderError) as e:
        rtc.Context(0)
    assert e.value.code == RT_ERR_NO_DEVICE


def test_product_path_does_not_import_the_oracle():
    pkg = os.path.join(PKG, "rtc_amd")
    for root, _, files in os.walk(os.path.join(PKG)):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                text = open(os.path.join(root, f), errors="replace").read()
                assert "pyoracle" not in text and "rtc_oracle" not in text and "liboracle" not in text, \
                    f"{os.path.relpath(os.path.join(root, f), ROOT)} references the oracle"
    assert os.path.isdir(pkg)
