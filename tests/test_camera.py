"""The product's host camera precompute (rt_camera_make / rt_camera_resize /
rt_camera_set_transform, csrc/scene_loader.cpp + host_math.hpp) against the
reference's own camera known answers (camera.rs:160-213) — not against the
oracle's camera, so a host camera bug cannot hide behind a shared input.
The device half (ray_for_pixel) is tests/test_gpu_kats.py."""
import json
import math
import os

from conftest import GOLDEN

GOLD = json.load(open(os.path.join(GOLDEN, "reference_kats.json")))["cases"]


def test_pixel_size_horizontal_and_vertical(rtc):
    # camera.rs:172-182 (assert_eq!)
    for w, h, name in ((200, 125, "camera.pixel_size_horizontal"), (125, 200, "camera.pixel_size_vertical")):
        cam = rtc.camera_make(w, h, math.pi / 2.0, (0, 0, 0), (0, 0, -1), (0, 1, 0))
        assert cam.pixel_size == GOLD[name]["expected"][0] == 0.009999999999999998
        assert (cam.width, cam.height, cam.field_of_view) == (w, h, math.pi / 2.0)


def test_resize_equals_a_fresh_camera(rtc):
    a = rtc.camera_make(160, 120, 1.05, (0, 1.5, -5), (0, 1, 0), (0, 1, 0))
    b = rtc.camera_resize(rtc.camera_make(7, 3, 1.05, (0, 1.5, -5), (0, 1, 0), (0, 1, 0)), 160, 120)
    for f in ("width", "height", "half_width", "half_height", "pixel_size"):
        assert getattr(a, f) == getattr(b, f), f
    assert list(a.inverse) == list(b.inverse) and list(a.origin) == list(b.origin)


def test_set_transformation_origin(rtc):
    # camera.rs:203-213: rotation_y(PI/4) * translation(0, -2, 5) -> origin (0, 2, -5) (assert_eq!)
    from rtc_amd import world as W
    cam = rtc.camera_make(201, 101, math.pi / 2.0, (0, 0, 0), (0, 0, -1), (0, 1, 0))
    t = rtc.camera_set_transform(cam, W.mat_mul(W.rotation_y(math.pi / 4.0), W.translation(0, -2, 5)))
    assert tuple(t.origin) == (0.0, 2.0, -5.0)
    ident = rtc.camera_set_transform(cam, W.IDENTITY)
    assert list(ident.inverse) == [1.0 if i % 5 == 0 else 0.0 for i in range(16)]
    assert tuple(ident.origin) == (0.0, 0.0, 0.0)
