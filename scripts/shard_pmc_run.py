#!/usr/bin/env python3
"""Workload for PMC passes over a frame split in row-block shards on one GPU
(VERDICT r5 items 1 and 7): WARM warm-up rounds, then ROUNDS
rounds that each render every shard of an N-way split of `scene` at W x H
once (u8, depth 6, the per-scene kernels as a warm renderer runs them).
rocprofv3 then sees ROUNDS x N timed tracer dispatches at the end;
scripts/shard_pmc_summary.py sums them per round, so N = 1 gives the whole
frame and N = 8 the eight shards a rank each renders at 8 GPUs.
Usage: python scripts/shard_pmc_run.py scene N [W H ROUNDS WARM]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

name, n = sys.argv[1], int(sys.argv[2])
w, h = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (3840, 2160)
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 5
warm = int(sys.argv[6]) if len(sys.argv) > 6 else 4
scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
cam = rtc_amd.camera_resize(scene.camera, w, h)
s = torch.cuda.current_stream()
with rtc_amd.Context(0) as ctx:
    ctx.set_jit(rtc_amd.RT_JIT_SYNC)
    ctx.upload(scene)
    rows = rtc_amd.shard_rows(h, n)
    out = torch.empty((rows, w, 3), dtype=torch.uint8, device="cuda")
    for _ in range(warm + rounds):
        for k in range(n):
            ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, n))
        torch.cuda.synchronize()
    print(f"{name} {w}x{h} shards={n}: {rounds} rounds after {warm} warm", flush=True)
