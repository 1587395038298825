"""Predicted multi-GPU render time per rank from one GPU: the kernel time of
each row-block shard of a frame (what rank s renders at N = shards), warm
(cost-ordered) launches, median of 5.  Diagnostic for DESIGN.md §6.
SHARD_INFLIGHT=F (round 6) adds, per shard, the time per frame of 40
consecutive frames of that shard with F frames in flight (F contexts
alternating on their own streams, as bench.py runs them)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

name, w, h = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("cover", 3840, 2160)
COUNTS = [int(x) for x in os.environ.get("SHARD_COUNTS", "1,2,4,8").split(",")]
scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
cam = rtc_amd.camera_resize(scene.camera, w, h)
s = torch.cuda.current_stream()
INFLIGHT = int(os.environ.get("SHARD_INFLIGHT", "1"))
streams = [torch.cuda.Stream() for _ in range(INFLIGHT)]
others = []
for _ in range(INFLIGHT if INFLIGHT > 1 else 0):
    c = rtc_amd.Context(0)
    c.set_jit(rtc_amd.RT_JIT_SYNC)
    c.set_frames_in_flight(INFLIGHT)  # (rtc.h planning hint, as bench.py sets it)
    c.upload(scene)
    others.append(c)
with rtc_amd.Context(0) as ctx:
    ctx.set_jit(rtc_amd.RT_JIT_SYNC)  # the per-scene kernels from the first frame (as a warm renderer runs)
    ctx.upload(scene)
    for shards in COUNTS:
        rows = rtc_amd.shard_rows(h, shards)
        out = torch.empty((rows, w, 3), dtype=torch.uint8, device="cuda")
        times = []
        for k in range(shards):
            for _ in range(3):
                ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, shards))
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, shards))
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            times.append(float(np.median(ts)))
        print(f"{name} {w}x{h} shards={shards}: per-shard ms " + " ".join(f"{t:.3f}" for t in times)
              + f"  max {max(times):.3f}  ideal {times[0] * 0 + sum(times) / shards:.3f}", flush=True)
        if INFLIGHT > 1:
            pipe = []
            for k in range(shards):
                outs = [torch.empty((rows, w, 3), dtype=torch.uint8, device="cuda") for _ in others]

                def frame(j):
                    i = j % INFLIGHT
                    others[i].render_device(cam, outs[i].data_ptr(), streams[i].cuda_stream, 6, "f32", "u8",
                                            (k, shards))
                for j in range(3 * INFLIGHT):
                    frame(j)
                torch.cuda.synchronize()
                reps = []
                for _ in range(5):
                    t0 = time.perf_counter()
                    for j in range(40):
                        frame(j)
                    torch.cuda.synchronize()
                    reps.append((time.perf_counter() - t0) * 1e3 / 40)
                pipe.append(float(np.median(reps)))
            print(f"{name} {w}x{h} shards={shards} inflight={INFLIGHT}: per-shard ms per frame "
                  + " ".join(f"{t:.3f}" for t in pipe) + f"  max {max(pipe):.3f}", flush=True)
