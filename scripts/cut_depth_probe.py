"""Timing experiment for the round-5 verdict's wavefront proposal (DESIGN.md
§6): how fast would an 8-way shard's pool launch be if the urgent (heavy)
items handed their deep generations to another kernel?  Run with
RTC_DEBUG=jit_flags=-DRTC_EXP_CUT_DEPTH=K, the per-scene pool kernel drops
the children at depth >= K of items with a priority (the frames are wrong);
this prints the slowest shard's kernel ms (warm, median of 5) and the
radiance rays per frame that the cut removed, i.e. what a drain kernel would
have to trace.  One JSON line per scene."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

SHARDS = int(os.environ.get("SHARDS", "8"))
s = torch.cuda.current_stream()
for name in sys.argv[1:] or ["cover", "table"]:
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
    cam = rtc_amd.camera_resize(scene.camera, 3840, 2160)
    with rtc_amd.Context(0) as ctx:
        ctx.set_jit(rtc_amd.RT_JIT_SYNC)
        ctx.upload(scene)
        rows = rtc_amd.shard_rows(2160, SHARDS)
        out = torch.empty((rows, 3840, 3), dtype=torch.uint8, device="cuda")
        times, rays = [], 0
        for k in range(SHARDS):
            for _ in range(3):
                ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, SHARDS))
            torch.cuda.synchronize()
            c0 = ctx.counters()["rays"]
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, SHARDS))
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            rays += (ctx.counters()["rays"] - c0) / 5
            times.append(float(np.median(ts)))
        print(json.dumps({"scene": name, "debug": os.environ.get("RTC_DEBUG", ""), "shards": SHARDS,
                          "slowest_ms": round(max(times), 4), "mean_ms": round(float(np.mean(times)), 4),
                          "rays_per_frame": int(rays), "jit_used": ctx.jit_status()["used"]}), flush=True)
