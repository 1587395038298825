"""The GPU kernels skip the hit's own shape in a shadow test when every lane of
the wave sits on that shape, the shape is flat (plane, triangle) or convex
(sphere, cube) and seen from outside, and the light is on the normal's side
(rtc_kernels.hip shade_ray / any_hit).  Geometrically that shape cannot block
the ray: the over point lies beyond the plane that supports the shape at the
hit and the ray moves away from it.  This checks the claim on the reference's
own algorithm: the f64 oracle built with ORC_CHECK_SELF_SHADOW counts, over
every shadow test of every reference scene, the eligible tests in which the
hit's own shape is the only blocker it finds.  There must be none, so the
f64 parity path (which must match the reference exactly) loses nothing.
CPU only (oracle/_build/liboracle_selfcheck.so)."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT, scene_fixture

SCENES = ["three_sphere_scene", "shadow_puppets", "reflect_refract", "refraction", "cover", "table", "metal",
          "cylinders"]


@pytest.fixture(scope="module")
def selfcheck():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    path = os.path.join(pyoracle.BUILD, "liboracle_selfcheck.so")
    if not os.path.exists(path):
        pyoracle.build()
    r = pyoracle._structs()
    L = C.CDLL(path)
    P = C.POINTER
    tabs = [P(r.ShapeDesc), C.c_uint32, P(r.MaterialDesc), C.c_uint32, P(r.PatternDesc), C.c_uint32,
            P(r.LightDesc), C.c_uint32]
    L.orc_render.argtypes = tabs + [P(r.CameraDesc), C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, P(C.c_double),
                                    P(r.Stats)]
    L.orc_render.restype = C.c_int
    L.orc_self_shadow_counts.argtypes = [P(C.c_uint64), P(C.c_uint64)]
    L.orc_self_shadow_counts.restype = C.c_int
    return L, r


def test_hit_shape_never_blocks_its_own_outer_shadow_ray(selfcheck, rtc):
    L, r = selfcheck
    for name in SCENES:
        scene = scene_fixture(name)
        cam = rtc.camera_resize(scene.camera, 192, 108)
        out = np.zeros((cam.height, cam.width, 3), dtype=np.float64)
        st = r.Stats()
        assert L.orc_render(*scene.args(), C.byref(cam), 6, 0, cam.height, 8,
                            out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)) == 0, name
    checked, violations = C.c_uint64(0), C.c_uint64(0)
    L.orc_self_shadow_counts(C.byref(checked), C.byref(violations))
    assert checked.value > 50_000, checked.value  # eligible shadow tests seen over the scenes
    assert violations.value == 0, f"{violations.value} of {checked.value} eligible shadow tests blocked by the hit shape only"
