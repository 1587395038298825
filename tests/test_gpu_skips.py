"""The acceleration-only skips change nothing, on the device, in f32 and f64.

any_hit (rtc_kernels.hip) skips work the reference does (world.rs:98-112
traces every shadow ray against every shape): the shadow ray of a light behind
the surface, planes with both ends of the segment on one side, cubes with a
face plane separating the segment or holding both ends, and the remaining
clusters once every lane is blocked; closest_hit takes a cube that holds a
light and every origin by its exit face.  RT_FLAG_NO_SKIPS turns all of them
off (the generic kernels at run time, the per-scene kernel through a build of
its own), so the frame without them must equal the product frame bit for bit,
counters included, on every reference scene and at 4K on table and cover, in
both precisions.  (The f32 skips were pinned only by a numpy model of the
kernel's arithmetic before: tests/test_shadow_skips.py.)
"""
import numpy as np
import pytest

from conftest import scene_fixture
from test_gpu_parity import SCENES, _counts

pytestmark = pytest.mark.gpu


def _both(ctx, rtc, cam, precision):
    a, sa = ctx.render(cam, 6, precision=precision)
    b, sb = ctx.render(cam, 6, precision=precision, flags=rtc.RT_FLAG_NO_SKIPS)
    return a, sa, b, sb


@pytest.mark.parametrize("precision,jit", [("f32", "sync"), ("f32", "off"), ("f64", "off")])
@pytest.mark.parametrize("name", SCENES)
def test_skips_are_exact_320x200(gpu_ctx, rtc, name, precision, jit):
    """jit=sync: the per-scene kernel the bench times against its no-skips
    build; jit=off: the generic kernel with and without the launch flag."""
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 320, 200)
    gpu_ctx.upload(scene)
    gpu_ctx.set_jit(rtc.RT_JIT_SYNC if jit == "sync" else rtc.RT_JIT_OFF)
    try:
        a, sa, b, sb = _both(gpu_ctx, rtc, cam, precision)
    finally:
        gpu_ctx.set_jit(rtc.RT_JIT_AUTO)
    assert np.array_equal(a, b), f"{name} {precision}: the skips changed {int((a != b).any(axis=2).sum())} px"
    assert _counts(sa) == _counts(sb)


@pytest.mark.parametrize("name", ["table", "cover"])
def test_skips_are_exact_4k_f32(gpu_ctx, rtc, name):
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 3840, 2160)
    gpu_ctx.upload(scene)
    gpu_ctx.set_jit(rtc.RT_JIT_SYNC)
    try:
        a, sa, b, sb = _both(gpu_ctx, rtc, cam, "f32")
        assert gpu_ctx.jit_status()["used"]
    finally:
        gpu_ctx.set_jit(rtc.RT_JIT_AUTO)
    assert np.array_equal(a, b), f"{name}: the skips changed {int((a != b).any(axis=2).sum())} px"
    assert _counts(sa) == _counts(sb)
