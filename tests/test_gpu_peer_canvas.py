"""The peer canvas (rtc.h rt_canvas_*) across two processes on the one GPU.

The multi-GPU tile split can assemble a frame without the RCCL gather: every
shard stores its pixels at their image rows into rank 0's canvas through an
IPC mapping, raises a completion flag, and waits for rank 0's release of the
previous frame before overwriting it (SURVEY.md §8e's gather, done as remote
stores).  RCCL refuses two ranks on one device, but two processes can share
an IPC handle there, so the protocol runs here end to end: this process owns
the canvas and renders shard 0, a child process maps it and renders shard 1,
for several frames in a row; each assembled frame must equal the single-GPU
frame bit for bit (cover at 3840x2160, u8, as the tiled bench gathers it).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import scene_fixture

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CHILD = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ray-tracer-challenge-rs_amd"))
import torch
import rtc_amd
from rtc_amd import scene_io
req = json.loads(sys.stdin.readline())
scene = scene_io.load(req["scene"])
cam = rtc_amd.camera_resize(scene.camera, req["w"], req["h"])
ctx = rtc_amd.Context(0)
ctx.upload(scene)
canvas = ctx.canvas_open(bytes.fromhex(req["handle"]), req["bytes"], req["shards"])
print("mapped", flush=True)
for seq in range(1, req["frames"] + 1):
    for shard in req["mine"]:
        ctx.render_to_canvas(cam, canvas, seq, req["depth"], "f32", req["out"], (shard, req["shards"]),
                             timeout_ms=60000.0)
torch.cuda.synchronize()
ctx.counters()  # raises on a peer-canvas timeout
print("rendered", flush=True)
sys.stdin.readline()  # the owner has read its last frame: unmap
ctx.canvas_close(canvas)
ctx.close()
print("closed", flush=True)
"""


def _run_split(gpu_ctx, rtc, name, w, h, out, frames, shards, child_shards):
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, w, h)
    gpu_ctx.upload(scene)
    dtype = np.uint8 if out == "u8" else np.float32
    ref, _ = gpu_ctx.render(cam, 6, precision="f32", out_format=out)
    nbytes = ref.nbytes
    canvas, handle = gpu_ctx.canvas_create(nbytes, shards)
    env = dict(os.environ)
    child = subprocess.Popen([sys.executable, "-c", CHILD, ROOT], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, text=True, env=env)
    try:
        child.stdin.write(json.dumps({
            "scene": os.path.join(HERE, "golden", "scenes", f"{name}.json"), "w": w, "h": h, "depth": 6, "out": out,
            "handle": handle.hex(), "bytes": nbytes, "shards": shards, "mine": child_shards, "frames": frames}) + "\n")
        child.stdin.flush()
        assert child.stdout.readline().strip() == "mapped", child.stderr.read()[-3000:]
        mine = [s for s in range(shards) if s not in child_shards]
        for seq in range(1, frames + 1):
            for shard in mine:
                gpu_ctx.render_to_canvas(cam, canvas, seq, 6, "f32", out, (shard, shards), timeout_ms=60000.0)
            gpu_ctx.canvas_wait(canvas, seq, timeout_ms=60000.0)
            img = gpu_ctx.canvas_read(canvas, ref.shape, dtype)
            assert np.array_equal(img, ref), f"frame {seq}: {int((img != ref).any(axis=2).sum())} px differ"
            gpu_ctx.canvas_release(canvas, seq)
        assert child.stdout.readline().strip() == "rendered", child.stderr.read()[-3000:]
        child.stdin.write("\n")
        child.stdin.flush()
        assert child.wait(timeout=120) == 0, child.stderr.read()[-3000:]
    finally:
        if child.poll() is None:
            child.kill()
            child.wait()
        gpu_ctx.canvas_close(canvas)


def test_two_processes_assemble_cover_4k(gpu_ctx, rtc):
    _run_split(gpu_ctx, rtc, "cover", 3840, 2160, "u8", frames=3, shards=2, child_shards=[1])


def test_two_processes_eight_shards_f32(gpu_ctx, rtc):
    """Eight shards over two processes (the child renders the odd ones), f32 canvas, ragged size."""
    _run_split(gpu_ctx, rtc, "reflect_refract", 333, 201, "real", frames=2, shards=8, child_shards=[1, 3, 5, 7])


def test_render_to_canvas_validates(gpu_ctx, rtc):
    scene = scene_fixture("three_sphere_scene")
    cam = rtc.camera_resize(scene.camera, 64, 32)
    gpu_ctx.upload(scene)
    canvas, _ = gpu_ctx.canvas_create(64 * 32 * 3, 2, ipc=False)
    try:
        with pytest.raises(rtc.RenderError):  # an f32 frame does not fit a u8-sized canvas
            gpu_ctx.render_to_canvas(cam, canvas, 1, 6, "f32", "real", (0, 2))
        with pytest.raises(rtc.RenderError):  # shard without a flag
            gpu_ctx.render_to_canvas(cam, canvas, 1, 6, "f32", "u8", (2, 3))
        for shard in (0, 1):
            gpu_ctx.render_to_canvas(cam, canvas, 1, 6, "f32", "u8", (shard, 2))
        gpu_ctx.canvas_wait(canvas, 1)
        ref, _ = gpu_ctx.render(cam, 6, precision="f32", out_format="u8")
        assert np.array_equal(gpu_ctx.canvas_read(canvas, ref.shape), ref)
    finally:
        gpu_ctx.canvas_close(canvas)


OPEN_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ray-tracer-challenge-rs_amd"))
import rtc_amd
req = json.loads(sys.stdin.readline())
ctx = rtc_amd.Context(0)
res = []
for nbytes, n_flags in req["tries"]:
    try:
        c = ctx.canvas_open(bytes.fromhex(req["handle"]), nbytes, n_flags)
        ctx.canvas_close(c)
        res.append("ok")
    except rtc_amd.RenderError as e:
        res.append(e.code)
ctx.close()
print(json.dumps(res), flush=True)
"""


def test_canvas_open_checks_the_creators_sizes(gpu_ctx, rtc):
    """rt_canvas_open reads the canvas's trailer (image bytes, flag count) and
    refuses sizes that differ from the creator's (a wrong
    `bytes` would have put the opener's flags at a wrong offset)."""
    nbytes, shards = 3840 * 2160 * 3, 8
    canvas, handle = gpu_ctx.canvas_create(nbytes, shards)
    try:
        tries = [(nbytes, shards), (nbytes - 256, shards), (nbytes + 4096, shards), (nbytes, shards - 1),
                 (nbytes * 2, shards)]
        r = subprocess.run([sys.executable, "-c", OPEN_CHILD, ROOT], input=json.dumps(
            {"handle": handle.hex(), "tries": tries}) + "\n", capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-3000:]
        got = json.loads(r.stdout.strip().splitlines()[-1])
        assert got[0] == "ok" and got[1:] == [rtc.RT_ERR_INVALID] * 4, got
    finally:
        gpu_ctx.canvas_close(canvas)
