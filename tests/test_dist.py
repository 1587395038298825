"""Multi-rank plumbing of the render path on CPU (gloo, world_size 2):
row-block sharding, the strip gather and the de-interleave that bench.py's
tiled mode runs over RCCL, plus the frames-mode job totals.

The oracle stands in for the device renderer here (test infrastructure
only): each rank renders exactly the canvas rows of its strip, so the
assembled frame must equal the full-frame render bit for bit.
"""
import os
import socket

import numpy as np
import pytest

from conftest import scene_fixture


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _render_strip(oracle, scene, cam, rows):
    strip = np.zeros((len(rows), cam.width, 3))
    y = 0
    while y < len(rows):
        if rows[y] < 0:
            y += 1
            continue
        y1 = y
        while y1 < len(rows) and rows[y1] == rows[y] + (y1 - y):
            y1 += 1
        strip[y:y1], _ = oracle.render(scene, cam, 6, rows=(int(rows[y]), int(rows[y1 - 1]) + 1))
        y = y1
    return strip


def _worker(rank, world, port, name, w, h, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import pyoracle
    import rtc_amd
    from rtc_amd import dist as rdist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene = scene_fixture(name)
        cam = rtc_amd.camera_resize(scene.camera, w, h)
        rows = rdist.strip_canvas_rows(h, world, rank)
        strip = torch.from_numpy(_render_strip(pyoracle, scene, cam, rows))
        gathered = torch.empty((world * len(rows), w, 3), dtype=torch.float64) if rank == 0 else None
        rdist.gather_strips(strip, gathered, world, rank)
        elapsed, rays = rdist.job_totals(1.0 + rank, 100.0 * (rank + 1), "cpu")
        if rank == 0:
            image = rdist.assemble_host(gathered.numpy(), h, world)
            np.savez(out_path, image=image, elapsed=elapsed, rays=rays)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,w,h", [("cover", 48, 37), ("three_sphere_scene", 40, 24)])
def test_tiled_gather_reassembles_the_frame(tmp_path, oracle, rtc, name, w, h):
    import torch.multiprocessing as mp
    world = 2
    out = str(tmp_path / "frame.npz")
    mp.spawn(_worker, args=(world, _free_port(), name, w, h, out), nprocs=world, join=True)
    res = np.load(out)
    scene = scene_fixture(name)
    ref, _ = oracle.render(scene, rtc.camera_resize(scene.camera, w, h), 6)
    assert np.array_equal(res["image"], ref)
    assert float(res["elapsed"]) == 2.0 and float(res["rays"]) == 300.0  # max time, summed rays


@pytest.mark.parametrize("h,shards", [(1, 1), (5, 2), (37, 3), (1080, 8), (2160, 8), (7, 8)])
def test_strip_rows_partition_the_canvas(h, shards):
    from rtc_amd import dist as rdist
    seen = np.concatenate([rdist.strip_canvas_rows(h, shards, s) for s in range(shards)])
    assert sorted(seen[seen >= 0].tolist()) == list(range(h))
    assert all(len(rdist.strip_canvas_rows(h, shards, s)) == rdist.strip_height(h, shards) for s in range(shards))


def test_assemble_host_inverts_the_split():
    from rtc_amd import dist as rdist
    h, w, shards = 29, 5, 3
    img = np.arange(h * w * 3, dtype=np.float32).reshape(h, w, 3)
    strips = []
    for s in range(shards):
        rows = rdist.strip_canvas_rows(h, shards, s)
        st = np.full((len(rows), w, 3), -1.0, dtype=np.float32)
        st[rows >= 0] = img[rows[rows >= 0]]
        strips.append(st)
    assert np.array_equal(rdist.assemble_host(np.concatenate(strips), h, shards), img)


@pytest.mark.parametrize("name", ["three_sphere_scene", "cover", "table", "reflect_refract"])
def test_scene_bytes_round_trip(name):
    from rtc_amd import dist as rdist
    scene = scene_fixture(name)
    data = rdist.scene_to_bytes(scene)
    back = rdist.scene_from_bytes(data)
    assert back.counts == scene.counts and back.duplicate_shapes == scene.duplicate_shapes
    assert rdist.scene_to_bytes(back) == data  # raw f64 fields: bit-exact
    with pytest.raises(ValueError):
        rdist.scene_from_bytes(data[:-1])


def _bcast_worker(rank, world, port, name, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from rtc_amd import dist as rdist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene = scene_fixture(name) if rank == 0 else None
        got = rdist.broadcast_scene(scene, rank, "cpu")
        with open(f"{out_path}.{rank}", "wb") as f:
            f.write(rdist.scene_to_bytes(got))
    finally:
        dist.destroy_process_group()


def test_broadcast_scene_from_rank0(tmp_path):
    """only rank 0 holds the world; every rank uploads the same tables."""
    import torch.multiprocessing as mp

    from rtc_amd import dist as rdist
    world = 2
    out = str(tmp_path / "scene")
    mp.spawn(_bcast_worker, args=(world, _free_port(), "cover", out), nprocs=world, join=True)
    ref = rdist.scene_to_bytes(scene_fixture("cover"))
    for r in range(world):
        assert open(f"{out}.{r}", "rb").read() == ref


def _camera_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import rtc_amd
    from rtc_amd import dist as rdist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cam = rtc_amd.camera_resize(scene_fixture("cover").camera, 3840, 2160) if rank == 0 else None
        got = rdist.share_camera(cam, rank)
        with open(f"{out_path}.{rank}", "wb") as f:
            f.write(bytes(got))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_camera_reaches_every_rank_bit_exact(tmp_path, rtc):
    """bench.py's tiled mode: the world stays on rank 0 (librtc broadcasts it),
    the camera goes to the other ranks over the control-plane group, raw."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "cam")
    mp.spawn(_camera_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    ref = bytes(rtc.camera_resize(scene_fixture("cover").camera, 3840, 2160))
    for r in range(2):
        assert open(f"{out}.{r}", "rb").read() == ref


def _fail_worker(rank, world, port, out_path, kind="render"):
    """Rank 1's upload fails (a malformed table: RT_ERR_INVALID from the
    library's validation, stood in for here since a group context needs GPUs);
    the step's status agreement must make every rank raise, then a later
    collective must still complete (nobody is left inside the failed step)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import rtc_amd
    from rtc_amd import dist as rdist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def upload():
            if rank == 1 and kind == "render":
                raise rtc_amd.RenderError(rtc_amd.RT_ERR_INVALID, "shape 3: material index out of range")
            if rank == 1:
                raise OSError("scene file vanished")  # not a RenderError
            return "uploaded"
        try:
            rdist.collective_call(upload, rank)
            code = 0
        except rtc_amd.RenderError as e:
            code = e.code
        except OSError:
            code = 99
        t = torch.tensor([1.0])
        dist.all_reduce(t)  # the group is still usable
        with open(f"{out_path}.{rank}", "w") as f:
            f.write(f"{code} {t.item()}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["render", "os"])
def test_a_rank_failing_its_upload_fails_every_rank(tmp_path, kind):
    import time

    import torch.multiprocessing as mp
    world = 2
    out = str(tmp_path / "status")
    t0 = time.monotonic()
    ctx = mp.spawn(_fail_worker, args=(world, _free_port(), out, kind), nprocs=world, join=False)
    while not ctx.join(timeout=5):
        assert time.monotonic() - t0 < 120, "a rank is still waiting after another failed its upload"
    codes = [open(f"{out}.{r}").read().split() for r in range(world)]
    # the failing rank re-raises its own exception: RT_ERR_INVALID, or the OSError
    assert int(codes[1][0]) == (-1 if kind == "render" else 99)
    assert int(codes[0][0]) == -8            # RT_ERR_COMM on the others
    assert all(float(c[1]) == 2.0 for c in codes)
