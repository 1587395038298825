#!/usr/bin/env python3
"""Diagnostic: host-side cost per frame launch (why wall ms/step > kernel ms).
Times K launches of the headline frame: (a) bare render_device loop,
(b) with torch events around each launch, (c) the raw ctypes call with
prebuilt arguments; plus a host-only loop that never waits on the GPU."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def main():
    import ctypes as C
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
    K = 400

    def run(label, body):
        for _ in range(20):
            body()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            body()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{label:32s} host {1e6 * (t1 - t0) / K:7.2f} us/launch   wall {1e6 * (t2 - t0) / K:7.2f} us/frame")

    run("render_device", lambda: ctx.render_device(cam, out.data_ptr(), sptr, 6, "f32"))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def with_events():
        ev[0].record(s)
        ctx.render_device(cam, out.data_ptr(), sptr, 6, "f32")
        ev[1].record(s)
    run("render_device + 2 torch events", with_events)
    opts = ctx.options(6, "f32")
    args = (ctx._h, C.byref(cam), C.byref(opts), C.c_void_p(out.data_ptr()), C.c_void_p(sptr))
    f = rtc_amd._lib.rt_render_device
    run("raw ctypes call", lambda: f(*args))
    ctx.close()


if __name__ == "__main__":
    main()
