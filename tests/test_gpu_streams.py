"""Launch ordering across streams (include/rtc.h conventions).

Every launch of a context shares its queue heads, per-tile costs and ray-pool
spill.  rt_render_device runs on the caller's stream and rt_render on the
context's own; a launch on a different stream than the previous one must
wait for the earlier stream's work, or the second launch's head reset could
land while the first is still claiming tiles (skipped or doubled tiles).
"""
import numpy as np
import pytest

from conftest import scene_fixture

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["reflect_refract", "three_sphere_scene"])
def test_render_device_on_side_stream_then_render(gpu_ctx, rtc, name):
    import torch
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 640, 400)
    gpu_ctx.upload(scene)
    ref, _ = gpu_ctx.render(cam, 6, precision="f32")
    side = torch.cuda.Stream()
    outs = [torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device="cuda") for _ in range(4)]
    for rnd in range(3):
        for o in outs:  # queued back to back on the side stream, no host sync
            gpu_ctx.render_device(cam, o.data_ptr(), side.cuda_stream, 6, "f32")
        img, _ = gpu_ctx.render(cam, 6, precision="f32")  # context stream, right away
        assert np.array_equal(img, ref), f"round {rnd}: host render differs"
        gpu_ctx.render_device(cam, outs[0].data_ptr(), torch.cuda.current_stream().cuda_stream, 6, "f32")
        torch.cuda.synchronize()
        for i, o in enumerate(outs):
            assert np.array_equal(o.cpu().numpy(), ref), f"round {rnd}: device render {i} differs"


@pytest.mark.parametrize("name", ["cover", "three_sphere_scene"])
def test_frames_in_flight_on_two_contexts(rtc, name):
    """bench.py's frames in flight: consecutive frames alternate between two
    contexts, each on a stream of its own, with no host sync in between (a
    frame's tail overlaps the next one's start).  Every frame equals the
    frame of one context rendering alone, and each context counts its own
    frames' rays."""
    import torch
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 640, 400)
    ctxs = [rtc.Context(0) for _ in range(2)]
    try:
        for c in ctxs:
            c.upload(scene)
        ref, st = ctxs[0].render(cam, 6, precision="f32")
        for c in ctxs:  # the planning hint (a throughput grid for the direct kernel): same frames
            c.set_frames_in_flight(2)
        streams = [torch.cuda.Stream() for _ in ctxs]
        outs = [torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device="cuda") for _ in ctxs]
        before = [c.counters()["rays"] for c in ctxs]
        for j in range(12):
            i = j % 2
            ctxs[i].render_device(cam, outs[i].data_ptr(), streams[i].cuda_stream, 6, "f32")
        torch.cuda.synchronize()
        for i, o in enumerate(outs):
            assert np.array_equal(o.cpu().numpy(), ref), f"context {i}"
        for i, c in enumerate(ctxs):
            assert c.counters()["rays"] - before[i] == 6 * st["rays"]
    finally:
        for c in ctxs:
            c.close()
