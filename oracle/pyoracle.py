"""TEST INFRASTRUCTURE — ctypes view of the f64 CPU oracle (oracle/_build/liboracle.so).

The oracle restates the reference's render path in C++ f64 (rtc_oracle.hpp)
and is pinned by the reference's own known answers (tests/test_oracle_kat.py).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline — never as the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(BUILD, "liboracle.so")
KAT = os.path.join(BUILD, "kat_runner")


def build(quiet: bool = True) -> None:
    """Compile the oracle with its Makefile (g++, -O3 -ffp-contract=off)."""
    subprocess.run(["make", "-C", HERE, "-j4"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def _structs():
    import importlib
    import sys
    pkg_dir = os.path.join(os.path.dirname(HERE), "ray-tracer-challenge-rs_amd")
    if pkg_dir not in sys.path:
        sys.path.insert(0, pkg_dir)
    return importlib.import_module("rtc_amd")


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        r = _structs()
        L = C.CDLL(LIB)
        P = C.POINTER
        tabs = [P(r.ShapeDesc), C.c_uint32, P(r.MaterialDesc), C.c_uint32, P(r.PatternDesc), C.c_uint32,
                P(r.LightDesc), C.c_uint32]
        L.orc_render.argtypes = tabs + [P(r.CameraDesc), C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                        P(C.c_double), P(r.Stats)]
        L.orc_render.restype = C.c_int
        L.orc_color_at.argtypes = tabs + [P(C.c_double), C.c_uint64, C.c_uint32, P(C.c_double), P(r.Stats)]
        L.orc_color_at.restype = C.c_int
        L.orc_camera.argtypes = [C.c_uint32, C.c_uint32, C.c_double, P(C.c_double), P(C.c_double), P(C.c_double),
                                 P(r.CameraDesc)]
        L.orc_camera.restype = C.c_int
        L.orc_inverse.argtypes = [P(C.c_double), P(C.c_double)]
        L.orc_inverse.restype = C.c_int
        L.orc_last_error.restype = C.c_char_p
        L.orc_last_generations.argtypes = [P(C.c_uint64), P(C.c_uint64)]
        L.orc_last_generations.restype = C.c_int
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError("oracle: " + lib().orc_last_error().decode())


def render(scene, camera=None, depth: int = 6, rows=None, threads: int = 1):
    """Camera::render (threads=1) / render_parallel: f64 canvas (rows, W, 3) + ray counters."""
    r = _structs()
    cam = camera if camera is not None else scene.camera
    r0, r1 = rows if rows is not None else (0, cam.height)
    out = np.zeros((r1 - r0, cam.width, 3), dtype=np.float64)
    st = r.Stats()
    _check(lib().orc_render(*scene.args(), C.byref(cam), depth, r0, r1, threads,
                            out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)))
    return out, st.as_dict()


def color_at(scene, rays, depth: int = 6):
    r = _structs()
    rays = np.ascontiguousarray(np.asarray(rays, dtype=np.float64).reshape(-1, 6))
    out = np.zeros((rays.shape[0], 3), dtype=np.float64)
    st = r.Stats()
    _check(lib().orc_color_at(*scene.args(), rays.ctypes.data_as(C.POINTER(C.c_double)), rays.shape[0], depth,
                              out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)))
    return out, st.as_dict()


def last_generations():
    """(traced, shaded) per `remaining` 0..16 of this thread's last render / color_at
    (a child ray runs at its parent's remaining - 1; the primary at the depth)."""
    t = np.zeros(17, dtype=np.uint64)
    s = np.zeros(17, dtype=np.uint64)
    _check(lib().orc_last_generations(t.ctypes.data_as(C.POINTER(C.c_uint64)), s.ctypes.data_as(C.POINTER(C.c_uint64))))
    return t, s


def camera(width, height, fov, frm, to, up):
    r = _structs()
    cam = r.CameraDesc()
    v = lambda x: (C.c_double * 3)(*map(float, x))  # noqa: E731
    _check(lib().orc_camera(width, height, float(fov), v(frm), v(to), v(up), C.byref(cam)))
    return cam


def inverse(m):
    a = (C.c_double * 16)(*np.asarray(m, dtype=np.float64).reshape(16))
    out = (C.c_double * 16)()
    _check(lib().orc_inverse(a, out))
    return np.array(out[:]).reshape(4, 4)


def quantize(img):
    """canvas.rs:117-123: round(clamp(c, 0, 1) * 255) as u8 (round half away from zero, NaN -> 0)."""
    c = np.nan_to_num(np.clip(img, 0.0, 1.0), nan=0.0) * 255.0
    t = np.trunc(c)
    return (t + (c - t >= 0.5)).astype(np.uint8)
