"""Rays per generation on the device (RT_FLAG_GENERATIONS, rt_read_generation_counts)
against the f64 oracle's counts of the reference recursion.

Generation g is `remaining` = depth - g (world.rs:70-86): the camera rays at
the depth, each reflected / refracted child one lower (world.rs:114-157).
f64 frames trace exactly the oracle's rays, so every generation's traced and
shaded counts are equal; the per-generation sums are the frame's rt_stats
(traced = primary + reflect + refract, shaded = shaded, and shadow = L x
shaded, world.rs:46-52).  The diagnostic frame's pixels equal a plain frame's.
"""
import numpy as np
import pytest

from conftest import scene_fixture

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,depth", [("reflect_refract", 6), ("cover", 6), ("table", 4), ("three_sphere_scene", 5)])
def test_generations_match_the_oracle(gpu_ctx, oracle, rtc, name, depth):
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 96, 64)
    gpu_ctx.upload(scene)
    img, st, gen = gpu_ctx.render_generations(cam, depth, precision="f64")
    plain, pst = gpu_ctx.render(cam, depth, precision="f64")
    assert np.array_equal(img, plain)
    ref, rst = oracle.render(scene, cam, depth, threads=8)
    t, s = oracle.last_generations()
    want_t = [int(t[depth - g]) for g in range(depth + 1)]
    want_s = [int(s[depth - g]) for g in range(depth + 1)]
    assert gen["traced"] == want_t and gen["shaded"] == want_s, (gen, want_t, want_s)
    assert sum(gen["traced"]) == st["primary"] + st["reflect"] + st["refract"]
    assert gen["traced"][0] == st["primary"] == cam.width * cam.height
    assert sum(gen["shaded"]) == st["shaded"] == rst["shaded"]
    assert st["shadow"] == len(scene.lights) * sum(gen["shaded"])


def test_generations_f32_frame_sums(gpu_ctx, rtc):
    """The f32 path (per-scene builds never take the flag: the generic kernel
    counts) sums to its own counters."""
    scene = scene_fixture("reflect_refract")
    cam = rtc.camera_resize(scene.camera, 320, 200)
    gpu_ctx.upload(scene)
    img, st, gen = gpu_ctx.render_generations(cam, 6, precision="f32")
    assert sum(gen["traced"]) == st["primary"] + st["reflect"] + st["refract"]
    assert sum(gen["shaded"]) == st["shaded"]
    assert gen["traced"][0] == 320 * 200 and gen["traced"][-1] > 0
