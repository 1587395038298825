"""Diagnostic: per-tile costs of a frame and of its 8-way
shards, with each launch's kernel time and per-workgroup stamps, saved for
offline scheduling simulations (scripts/shard_sim.py).
Usage: python scripts/shard_costs.py [scene] [W H] -> gpurun_out/costs_<scene>.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cover"
w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (3840, 2160)
scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
cam = rtc_amd.camera_resize(scene.camera, w, h)
s = torch.cuda.current_stream()
res = {}
with rtc_amd.Context(0) as ctx:
    ctx.upload(scene)
    for shards in (1, 8):
        rows = rtc_amd.shard_rows(h, shards)
        out = torch.empty((rows, w, 3), dtype=torch.uint8, device="cuda")
        for k in range(shards):
            for _ in range(6):
                ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, shards))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, shards))
            e1.record(s)
            torch.cuda.synchronize()
            res[f"ms_{shards}_{k}"] = np.array(e0.elapsed_time(e1))
            res[f"cost_{shards}_{k}"] = ctx.debug_tile_costs().copy()
            ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, shards), rtc_amd.RT_FLAG_STAMPS)
            torch.cuda.synchronize()
            res[f"stamps_{shards}_{k}"] = ctx.debug_stamps().copy()
            print(name, shards, k, float(res[f"ms_{shards}_{k}"]), len(res[f"cost_{shards}_{k}"]),
                  float(res[f"cost_{shards}_{k}"].sum()) * 1e-5, flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"costs_{name}.npz"), **res)
