#!/usr/bin/env python3
"""GPU probe (not a test): do consecutive frames gain from running on two
streams (two contexts, frames alternating), so that one frame's launch
tail overlaps the next frame's start?  Host clock over K frames after a
warm-up, median of ROUNDS:
  three_sphere 1920x1080 f32 (configs[1], the direct kernel), K = 1000
  cover 3840x2160 u8, shard 0 of 8 (what one rank renders at N = 8), K = 200
Frames go to one output buffer per context; the last frame of each is
checked against the one-stream render.  Usage: overlap_probe.py [rounds]"""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402


def case(name, w, h, depth, out, shard, k, rounds):
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
    cam = rtc_amd.camera_resize(scene.camera, w, h)
    rows = rtc_amd.shard_rows(h, shard[1]) if shard[1] > 1 else h
    dt = torch.uint8 if out == "u8" else torch.float32
    ctxs = [rtc_amd.Context(0) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    bufs = [torch.empty((rows, w, 3), dtype=dt, device="cuda") for _ in range(2)]
    try:
        for c in ctxs:
            c.upload(scene)

        def f(i, s):
            ctxs[i].render_device(cam, bufs[i].data_ptr(), streams[s].cuda_stream, depth, "f32", out, shard)

        for i in range(2):
            f(i, i)
            f(i, i)
            ctxs[i].jit_wait(120000.0)
            for _ in range(50):
                f(i, i)
        torch.cuda.synchronize()
        one, two = [], []
        for _ in range(rounds):
            for _ in range(100):
                f(0, 0)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(k):
                f(0, 0)
            torch.cuda.synchronize()
            one.append((time.perf_counter() - t) * 1e3 / k)
            ref = bufs[0].clone()
            for _ in range(100):
                f(0, 0)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for j in range(k):
                f(j & 1, j & 1)
            torch.cuda.synchronize()
            two.append((time.perf_counter() - t) * 1e3 / k)
        same = bool(torch.equal(bufs[0], ref) and torch.equal(bufs[1], ref))
        print(json.dumps({"case": f"{name}@{w}x{h} shard {shard[0]}/{shard[1]}", "frames": k,
                          "one_stream_ms": statistics.median(one), "two_streams_ms": statistics.median(two),
                          "gain": statistics.median(one) / statistics.median(two), "frames_equal": same}), flush=True)
    finally:
        for c in ctxs:
            c.close()


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    torch.cuda.set_device(0)
    case("three_sphere_scene", 1920, 1080, 5, "real", (0, 1), 1000, rounds)
    case("cover", 3840, 2160, 6, "u8", (0, 8), 200, rounds)
    case("table", 3840, 2160, 6, "u8", (0, 8), 200, rounds)
    case("reflect_refract", 1920, 1080, 6, "real", (0, 1), 200, rounds)


if __name__ == "__main__":
    main()
