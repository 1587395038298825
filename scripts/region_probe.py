#!/usr/bin/env python3
"""GPU probe (not a test): what a K = 20 frame region costs beyond K frames.
configs[1] (three_sphere 1920x1080, depth 5, f32) on a side stream; each
round first runs 200 untimed frames and synchronizes, then one variant of
the region, host clock between synchronizes (as bench.py):
  plain    t0, K launches, sync
  events   t0, event, K launches, event, sync           (bench.py timed_launches)
  counters counters() (device sync + copy), then `events`
  idle1ms  1 ms of host sleep (GPU idle), then `events`
  idle10ms 10 ms of host sleep, then `events`
Median and min us per step over ROUNDS rounds, plus the 1000-frame rate.
Usage (GPU box): python scripts/region_probe.py [rounds]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def main():
    import torch

    import rtc_amd
    from rtc_amd import scene_io
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    k = 20
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", "three_sphere_scene.json"))
    cam = rtc_amd.camera_resize(scene.camera, 1920, 1080)
    ctx = rtc_amd.Context(0)
    ctx.upload(scene)
    img = torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()

    def step():
        ctx.render_device(cam, img.data_ptr(), s.cuda_stream, 5, "f32", "real")

    step()
    step()
    ctx.jit_wait(120000.0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    e1.record(s)
    for _ in range(2000):
        step()
    torch.cuda.synchronize()

    def region(events):
        t0 = time.perf_counter()
        if events:
            e0.record(s)
        for _ in range(k):
            step()
        if events:
            e1.record(s)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6 / k, (e0.elapsed_time(e1) * 1e3 / k if events else None)

    def pre(kind):
        if kind == "counters":
            ctx.counters()
        elif kind == "idle1ms":
            time.sleep(0.001)
        elif kind == "idle10ms":
            time.sleep(0.01)

    kinds = ["plain", "events", "counters", "idle1ms", "idle10ms"]
    res = {x: [] for x in kinds}
    dev = {x: [] for x in kinds}
    for _ in range(rounds):
        for kind in kinds:
            for _ in range(200):
                step()
            torch.cuda.synchronize()
            pre(kind)
            host, ev = region(kind != "plain")
            res[kind].append(host)
            if ev is not None:
                dev[kind].append(ev)
    t0 = time.perf_counter()
    for _ in range(1000):
        step()
    torch.cuda.synchronize()
    steady = (time.perf_counter() - t0) * 1e6 / 1000
    for kind in kinds:
        print(json.dumps({"region": kind, "steps": k, "host_us_per_step_median": statistics.median(res[kind]),
                          "host_us_per_step_min": min(res[kind]),
                          "event_us_per_step_median": statistics.median(dev[kind]) if dev[kind] else None,
                          "steady_1000_us_per_step": steady}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
