#!/usr/bin/env python3
"""Diagnostic: fixed cost of a short timed region (the driver's --steps 20).
After a 300 ms warm-up, times K=20 headline frames 15 times per variant:
  sync     : t0, event, K launches, event, torch.cuda.synchronize(), t1 (bench.py)
  evsync   : the same, e1.synchronize() before torch.cuda.synchronize()
  spin     : the same, busy-polling e1.query() first
and prints the median wall us/frame next to the event-bracket us/frame."""
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
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", "three_sphere_scene.json"))
    cam = rtc_amd.camera_resize(scene.camera, 1920, 1080)
    ctx = rtc_amd.Context(0)
    ctx.upload(scene)
    out = torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    sptr = s.cuda_stream
    K = int(os.environ.get("K", "20"))

    def step():
        ctx.render_device(cam, out.data_ptr(), sptr, 5, "f32")

    t = time.perf_counter()
    while time.perf_counter() - t < 0.3:
        for _ in range(100):
            step()
        torch.cuda.synchronize()

    def region(kind):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(s)
        for _ in range(K):
            step()
        e1.record(s)
        th = time.perf_counter()
        if kind == "evsync":
            e1.synchronize()
        elif kind == "spin":
            while not e1.query():
                pass
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        return 1e6 * (t1 - t0) / K, 1e3 * e0.elapsed_time(e1) / K, 1e6 * (th - t0) / K

    for kind in ("sync", "evsync", "spin", "sync"):
        r = [region(kind) for _ in range(15)]
        w = statistics.median(x[0] for x in r)
        e = statistics.median(x[1] for x in r)
        h = statistics.median(x[2] for x in r)
        print(f"{kind:8s} K={K} wall {w:6.2f} us/frame  events {e:6.2f} us/frame  host submit {h:5.2f} us/frame  "
              f"fixed {K * (w - e):6.1f} us", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
