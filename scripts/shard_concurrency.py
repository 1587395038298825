#!/usr/bin/env python3
"""Diagnostic: is the 8-way shard's extra
time work or an under-filled GPU?  On one GPU, event-timed (median of REPS):
  whole     the frame in one launch
  shards    each of the 8 shards alone (sum and max)
  serial8   the 8 shard launches back to back on one stream (one bracket)
  conc8     the 8 shard launches on 8 streams at once (one bracket)
If conc8 is close to `whole` while the sum of `shards` is not, a shard
launch on its own leaves the GPU partly idle (ramp, tail, heavy chains);
if conc8 is close to the sum, the shards do more work.  Per-scene kernels
(RT_JIT_SYNC), u8 canvas, depth 6.  Usage: shard_concurrency.py [scene ...]"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

REPS = 7
N = 8


def bracket(fn, streams):
    """ms from an event on streams[0] (after every stream joined it) to the
    last stream's end."""
    main = streams[0]
    e0 = torch.cuda.Event(enable_timing=True)
    ends = [torch.cuda.Event(enable_timing=True) for _ in streams]
    torch.cuda.synchronize()
    e0.record(main)
    for s in streams[1:]:
        s.wait_event(e0)
    fn()
    for s, e in zip(streams, ends):
        e.record(s)
    torch.cuda.synchronize()
    return max(e0.elapsed_time(e) for e in ends)


def main():
    scenes = sys.argv[1:] or ["cover", "table"]
    streams = [torch.cuda.Stream() for _ in range(N)]
    for name in scenes:
        scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
        cam = rtc_amd.camera_resize(scene.camera, 3840, 2160)
        # one context per shard: a context's launches share its queue heads,
        # tile costs and spill region, so it orders a launch on another
        # stream after its previous one (rtc_host.cpp order_after_last)
        ctxs = [rtc_amd.Context(0) for _ in range(N)]
        try:
            for c in ctxs:
                c.set_jit(rtc_amd.RT_JIT_SYNC)
                c.upload(scene)
            ctx = ctxs[0]
            full = torch.empty((2160, 3840, 3), dtype=torch.uint8, device="cuda")
            rows = rtc_amd.shard_rows(2160, N)
            outs = [torch.empty((rows, 3840, 3), dtype=torch.uint8, device="cuda") for _ in range(N)]
            whole_ctx = rtc_amd.Context(0)
            whole_ctx.set_jit(rtc_amd.RT_JIT_SYNC)
            whole_ctx.upload(scene)

            def whole():
                whole_ctx.render_device(cam, full.data_ptr(), streams[0].cuda_stream, 6, "f32", "u8")

            def shard(k, s):
                ctxs[k].render_device(cam, outs[k].data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, N))

            def serial8():
                for k in range(N):
                    shard(k, streams[0])

            def conc8():
                for k in range(N):
                    shard(k, streams[k])

            # warm every launch shape (each shard's tile costs and order are its own)
            for _ in range(4):
                whole()
                serial8()
            torch.cuda.synchronize()
            res = {"scene": name, "size": "3840x2160", "n": N}
            res["whole_ms"] = statistics.median(bracket(whole, streams[:1]) for _ in range(REPS))
            per = []
            for k in range(N):
                per.append(statistics.median(bracket(lambda: shard(k, streams[0]), streams[:1]) for _ in range(REPS)))
            res["shard_ms"] = [round(x, 4) for x in per]
            res["shard_sum_ms"] = sum(per)
            res["shard_max_ms"] = max(per)
            res["serial8_ms"] = statistics.median(bracket(serial8, streams[:1]) for _ in range(REPS))
            res["conc8_ms"] = statistics.median(bracket(conc8, streams) for _ in range(REPS))
            res["sum_over_whole"] = res["shard_sum_ms"] / res["whole_ms"]
            res["conc8_over_whole"] = res["conc8_ms"] / res["whole_ms"]
            print(json.dumps(res), flush=True)
            whole_ctx.close()
        finally:
            for c in ctxs:
                c.close()


if __name__ == "__main__":
    main()
