"""BASELINE configs[0]: scenes/three_sphere_scene.yaml at 320x240 in serial CPU
mode (Camera::render, camera.rs:79-95), the reference's own CPU-runnable case.

The oracle's serial restatement of Camera::render and its render_parallel
restatement (camera.rs:97-112) give the same canvas bit for bit and the same
ray counters (pixels are independent; the reference's two modes differ only
in scheduling), and the frame traces exactly 2·W·H rays: every camera ray
meets a wall or the floor (three planes), and each shaded hit casts one
shadow ray to the scene's one light.  The GPU path at
this size is checked against the serial frame in tests/test_gpu_fullsize.py.
"""
import numpy as np

from conftest import scene_fixture

W, H = 320, 240


def test_config0_serial_equals_parallel(rtc, oracle):
    scene = scene_fixture("three_sphere_scene")
    cam = rtc.camera_resize(scene.camera, W, H)
    serial, st_s = oracle.render(scene, cam, 6, threads=1)
    parallel, st_p = oracle.render(scene, cam, 6, threads=4)
    assert serial.shape == (H, W, 3)
    assert np.array_equal(serial, parallel)
    assert st_s == st_p
    assert st_s["primary"] == W * H and st_s["shadow"] == W * H
    assert st_s["reflect"] == st_s["refract"] == 0 and st_s["rays"] == 2 * W * H


def test_config0_depth5_equals_depth6(rtc, oracle):
    """BASELINE quotes "reflection depth 5"; the scene has no reflective or
    transparent material, so depth 5 and the reference's 6 render the same."""
    scene = scene_fixture("three_sphere_scene")
    cam = rtc.camera_resize(scene.camera, W, H)
    a, sa = oracle.render(scene, cam, 5, threads=4)
    b, sb = oracle.render(scene, cam, 6, threads=4)
    assert np.array_equal(a, b) and sa == sb
