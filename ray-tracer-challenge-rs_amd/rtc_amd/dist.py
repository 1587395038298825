"""Multi-GPU plumbing of the render path.

Pixels are independent (camera.rs:106-110: every pixel is its own
`color_at`), so a frame splits into shards with one data exchange at the end:

* tiled (the north star's split, the library's own multi-GPU contexts,
  csrc/rtc_group.cpp): ONE frame is split into cyclic RT_TILE_H-row blocks
  (block t belongs to shard t % N, balancing rows of very different cost).
  Shard s renders its blocks, in order, into a contiguous strip of
  `strip_height` rows (strips are padded to equal height so the gather has one
  send count); librtc RCCL-gathers the strips to rank 0, which de-interleaves
  them on the device (rt_assemble_shards; `assemble_host` is its host mirror
  for tests).  The world is flattened on rank 0 and RCCL-broadcast by
  rt_scene_upload; this module only shares the communicator's unique id
  (`share_unique_id`) and the camera over the control-plane process group.
* frames (opt-in, weak scaling): each rank renders whole frames; a job's
  throughput is the rays of all ranks over the slowest rank's time
  (`job_totals`).  No collective touches the data path.

`gather_strips` / `broadcast_scene` are the same exchanges written with
torch.distributed; the gloo tests (tests/test_dist.py) run them on CPU.
"""
from __future__ import annotations

import numpy as np

from . import RT_TILE_H, shard_rows


def strip_height(height: int, shards: int) -> int:
    """Rows of every shard's strip (rt_shard_rows)."""
    return shard_rows(height, shards)


def strip_canvas_rows(height: int, shards: int, shard: int) -> np.ndarray:
    """Canvas row of each strip row of `shard`, in strip order; -1 marks the
    padding rows past the canvas (never read by the assembly)."""
    n_blocks = (height + RT_TILE_H - 1) // RT_TILE_H
    rows = np.full(strip_height(height, shards), -1, dtype=np.int64)
    k = 0
    for t in range(shard, n_blocks, shards):
        for w in range(RT_TILE_H):
            y = t * RT_TILE_H + w
            rows[k] = y if y < height else -1
            k += 1
    return rows


def assemble_host(gathered: np.ndarray, height: int, shards: int) -> np.ndarray:
    """Host mirror of rt_assemble_shards: gathered = shard-major strips
    (shards * strip_height, W, C) -> (height, W, C) image."""
    strip = strip_height(height, shards)
    image = np.empty((height,) + gathered.shape[1:], dtype=gathered.dtype)
    for s in range(shards):
        rows = strip_canvas_rows(height, shards, s)
        keep = rows >= 0
        image[rows[keep]] = gathered[s * strip:(s + 1) * strip][keep]
    return image


def gather_strips(strip, gathered, world: int, rank: int, dst: int = 0) -> None:
    """torch.distributed gather of equal-height strips to `dst`; `gathered`
    is the (world * strip_height, W, C) receive buffer on `dst` (None elsewhere)."""
    import torch.distributed as dist
    chunks = list(gathered.chunk(world)) if rank == dst else None
    dist.gather(strip, chunks, dst=dst)


_HEADER = np.dtype([("magic", "<u4"), ("version", "<u4"), ("n", "<u4", 4), ("duplicate_shapes", "<u4")])
_MAGIC = 0x52544353  # "SCTR"


def scene_to_bytes(scene) -> bytes:
    """The flattened world as one byte string: a header (table counts), then
    the raw POD tables rt_scene_upload takes and the camera, in that order."""
    from . import RT_ABI_VERSION
    hdr = np.zeros((), dtype=_HEADER)
    hdr["magic"], hdr["version"] = _MAGIC, RT_ABI_VERSION
    hdr["n"] = scene.counts
    hdr["duplicate_shapes"] = scene.duplicate_shapes
    parts = [hdr.tobytes()] + [bytes(t) for t in (scene.shapes, scene.materials, scene.patterns, scene.lights)]
    return b"".join(parts) + bytes(scene.camera)


def scene_from_bytes(data: bytes):
    """Inverse of scene_to_bytes (bit-exact: the f64 fields are copied raw)."""
    import ctypes as C

    from . import RT_ABI_VERSION, CameraDesc, LightDesc, MaterialDesc, PatternDesc, SceneTables, ShapeDesc
    hdr = np.frombuffer(data[:_HEADER.itemsize], dtype=_HEADER)[0]
    if hdr["magic"] != _MAGIC or hdr["version"] != RT_ABI_VERSION:
        raise ValueError("not a scene broadcast of this ABI version")
    off = _HEADER.itemsize
    tables = []
    for cls, n in zip((ShapeDesc, MaterialDesc, PatternDesc, LightDesc), hdr["n"]):
        arr = (cls * int(n))()
        size = C.sizeof(arr)
        C.memmove(arr, data[off:off + size], size)
        tables.append(arr)
        off += size
    cam = CameraDesc.from_buffer_copy(data[off:off + C.sizeof(CameraDesc)])
    if off + C.sizeof(CameraDesc) != len(data):
        raise ValueError("scene broadcast has the wrong length")
    return SceneTables(*tables, cam, int(hdr["duplicate_shapes"]))


def broadcast_scene(scene, rank: int, device, src: int = 0):
    """the world only `src` holds (as the reference's
    single caller does) goes to every rank: its length, then its bytes, as
    torch.distributed broadcasts (RCCL over xGMI for CUDA `device`, gloo for
    "cpu").  Every rank returns the same tables; `scene` is ignored off `src`."""
    import torch
    import torch.distributed as dist
    payload = scene_to_bytes(scene) if rank == src else b""
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    dist.broadcast(n, src=src)
    buf = (torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device) if rank == src
           else torch.empty(int(n.item()), dtype=torch.uint8, device=device))
    dist.broadcast(buf, src=src)
    return scene if rank == src else scene_from_bytes(buf.cpu().numpy().tobytes())


def job_totals(elapsed_s: float, rays: float, device) -> tuple[float, float]:
    """(max elapsed over ranks, sum of rays over ranks): the whole-job
    throughput is sum(rays) / max(elapsed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(elapsed_s), float(rays)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    r = torch.tensor([rays], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(r, op=dist.ReduceOp.SUM)
    return float(t.item()), float(r.item())


def share_unique_id(rank: int, src: int = 0) -> bytes:
    """The RCCL unique id of a librtc group (rt_comm_unique_id on `src`),
    sent to every rank over the initialised torch.distributed process group."""
    import torch.distributed as dist

    from . import comm_unique_id
    box = [comm_unique_id() if rank == src else None]
    dist.broadcast_object_list(box, src=src)
    return box[0]


def share_camera(camera, rank: int, src: int = 0):
    """The camera `src` holds, as raw bytes (bit-exact), to every rank."""
    import torch.distributed as dist

    from . import CameraDesc
    box = [bytes(camera) if rank == src else None]
    dist.broadcast_object_list(box, src=src)
    return CameraDesc.from_buffer_copy(box[0])


def collective_call(fn, rank: int, device="cpu"):
    """Run one rank's part of a collective librtc step (fn() on this rank)
    and agree on its outcome before anyone goes on: every rank contributes
    its status (0, the RenderError code it raised, or 1 for any other
    exception) to one all-reduce, and
    if any rank failed, every rank raises (the failing ones their own error,
    the others RT_ERR_COMM naming the first failing rank).  So a rank that
    fails its upload cannot leave the others waiting in the next collective
    (bench.py's tiled mode; the library's own group upload agrees the same
    way over RCCL, rtc_group.cpp)."""
    import torch
    import torch.distributed as dist

    from . import RT_ERR_COMM, RenderError
    err, result = None, None
    try:
        result = fn()
    except Exception as e:  # noqa: BLE001  (any failure must still reach the all-reduce)
        err = e
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        if err is not None:
            raise err
        return result
    world = dist.get_world_size()
    # per rank: 0 = ok, else -code (codes are negative): one MAX reduce of a world-long vector
    st = torch.zeros(world, dtype=torch.int64, device=device)
    # a RenderError contributes its code, anything else (a ValueError or
    # OSError of the Python upload path) a generic nonzero status
    code = int(getattr(err, "code", 0) or 0) if isinstance(err, RenderError) else -1
    st[rank] = 0 if err is None else max(1, -code)
    dist.all_reduce(st, op=dist.ReduceOp.MAX)
    if err is not None:
        raise err
    bad = [r for r in range(world) if int(st[r]) != 0]
    if bad:
        raise RenderError(RT_ERR_COMM, f"rank {bad[0]} failed this step (status {-int(st[bad[0]])}); "
                                       f"failed ranks: {bad}")
    return result
