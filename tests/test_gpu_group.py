"""Multi-GPU contexts of the C-ABI (rtc_group.cpp) on the one-GPU test box.

The RCCL path — the scene broadcast inside rt_scene_upload, the shard
render into a strip, ncclGather onto rank 0 and the de-interleave — runs
here with one rank, both as a one-process group (rt_context_create_multi,
ncclCommInitAll) and as a rank of a one-process-per-GPU group
(rt_context_create_rank, ncclCommInitRank).  Its frames must equal the
single-GPU context's bit for bit, counters included.  The N-rank row-block
math is pinned on CPU (tests/test_shards.py) and the 8-shard split on one
device against the single-shot frame (tests/test_gpu_fullsize.py).
"""
import numpy as np
import pytest

from conftest import scene_fixture

pytestmark = pytest.mark.gpu


def _counts(st):
    return {k: st[k] for k in ("primary", "shadow", "reflect", "refract", "shaded", "lit_patterned",
                               "refract_evals", "schlick_evals")}


@pytest.fixture(params=["multi", "rank"])
def group_ctx(request, rtc):
    if request.param == "multi":
        ctx = rtc.Context.multi([0])
    else:
        ctx = rtc.Context.rank(0, 1, 0, rtc.comm_unique_id())
    yield ctx
    ctx.close()


@pytest.mark.parametrize("gather", ["rccl", "peer"])
@pytest.mark.parametrize("name", ["cover", "three_sphere_scene", "reflect_refract"])
def test_group_frames_equal_single_gpu(gpu_ctx, group_ctx, rtc, name, gather):
    """Both ways of bringing the shards to rank 0: the RCCL gather of strips and
    the peer canvas (shards store at image rows, flags, release)."""
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 480, 270)
    assert group_ctx.group() == (1, 0, 1)
    group_ctx.set_gather(rtc.RT_GATHER_PEER if gather == "peer" else rtc.RT_GATHER_RCCL)
    group_ctx.upload(scene)
    gpu_ctx.upload(scene)
    for precision, fmt in (("f32", "real"), ("f64", "real"), ("f32", "u8")):
        a, sa = gpu_ctx.render(cam, 6, precision=precision, out_format=fmt)
        b, sb = group_ctx.render(cam, 6, precision=precision, out_format=fmt)
        assert np.array_equal(a, b), (name, precision, fmt)
        assert _counts(sa) == _counts(sb)
        assert sb["n_shards"] == 1 and sb["frame_ms"] >= sb["kernel_ms"] > 0 and sb["gather_ms"] >= 0


def test_group_render_device_and_options(gpu_ctx, group_ctx, rtc):
    import torch
    scene = scene_fixture("table")
    cam = rtc.camera_resize(scene.camera, 333, 201)  # ragged last tile row
    group_ctx.upload(scene)
    gpu_ctx.upload(scene)
    ref, _ = gpu_ctx.render(cam, 6, precision="f32")
    out = torch.zeros((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):  # repeated frames: cost-ordered pool launches, reused strips
        group_ctx.render_device(cam, out.data_ptr(), s, 6, "f32")
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    with pytest.raises(rtc.RenderError):  # the group shards frames itself
        group_ctx.render(cam, 6, precision="f32", shard=(0, 2))


def test_group_upload_errors_are_reported(group_ctx, rtc):
    bad = scene_fixture("cover")
    bad.shapes[0].material = 999
    with pytest.raises(rtc.RenderError):
        group_ctx.upload(bad)
    with pytest.raises(rtc.RenderError):  # nothing uploaded yet
        group_ctx.render(rtc.camera_resize(bad.camera, 8, 8), 6)


def test_group_back_to_back_frames(gpu_ctx, group_ctx, rtc):
    """Back-to-back render_device calls with nothing in between, of
    alternating cameras, sizes and formats into separate outputs on a torch
    side stream (strip and gather buffers reused and resized between frames):
    each must equal the single-GPU frame, and a host-path render queued right
    after must see its own frame."""
    import torch
    scene = scene_fixture("reflect_refract")
    group_ctx.upload(scene)
    gpu_ctx.upload(scene)
    cams = [rtc.camera_resize(scene.camera, 320, 180), rtc.camera_resize(scene.camera, 256, 200)]
    view = np.linalg.inv(np.array(list(cams[0].inverse)).reshape(4, 4))
    shift = np.array([[1, 0, 0, 0.3], [0, 1, 0, -0.2], [0, 0, 1, 0.5], [0, 0, 0, 1.0]])
    moved = rtc.camera_set_transform(cams[0], shift @ view)
    jobs = [(cams[0], "real"), (cams[1], "u8"), (moved, "real"), (cams[1], "real"), (cams[0], "u8"), (moved, "u8")]
    refs = [gpu_ctx.render(c, 6, precision="f32", out_format=f)[0] for c, f in jobs]
    side = torch.cuda.Stream()
    outs = []
    with torch.cuda.stream(side):
        for c, f in jobs:
            o = torch.zeros((c.height, c.width, 3), dtype=torch.uint8 if f == "u8" else torch.float32, device="cuda")
            group_ctx.render_device(c, o.data_ptr(), side.cuda_stream, 6, "f32", f)
            outs.append(o)
    host, _ = group_ctx.render(cams[1], 6, precision="f32")
    side.synchronize()
    for (c, f), o, r in zip(jobs, outs, refs):
        assert np.array_equal(o.cpu().numpy(), r), (c.width, c.height, f)
    assert np.array_equal(host, refs[3])


@pytest.mark.parametrize("gather", ["rccl", "peer"])
def test_two_group_contexts_in_flight(gpu_ctx, rtc, gather):
    """bench.py's tiled lines with frames in flight: two rank-form groups, each
    with its own communicator, stream and u8 canvas, rendering alternate
    frames with no host sync in between and the planning hint for two in
    flight.  Every frame equals the single-GPU context's."""
    import torch
    scene = scene_fixture("cover")
    cam = rtc.camera_resize(scene.camera, 640, 360)
    gpu_ctx.upload(scene)
    ref, _ = gpu_ctx.render(cam, 6, precision="f32", out_format="u8")
    ctxs = [rtc.Context.rank(0, 1, 0, rtc.comm_unique_id()) for _ in range(2)]
    try:
        for c in ctxs:
            c.set_gather(rtc.RT_GATHER_PEER if gather == "peer" else rtc.RT_GATHER_RCCL)
            c.upload(scene)
            c.set_frames_in_flight(2)
        streams = [torch.cuda.Stream() for _ in ctxs]
        outs = [torch.zeros((cam.height, cam.width, 3), dtype=torch.uint8, device="cuda") for _ in ctxs]
        for j in range(10):
            i = j % 2
            ctxs[i].render_device(cam, outs[i].data_ptr(), streams[i].cuda_stream, 6, "f32", "u8")
        torch.cuda.synchronize()
        for i, o in enumerate(outs):
            assert np.array_equal(o.cpu().numpy(), ref), f"group {i}"
    finally:
        for c in ctxs:
            c.close()
