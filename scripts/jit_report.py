#!/usr/bin/env python3
"""Diagnostic: which frames run a per-scene kernel (rt_jit_status) and, with
RTC_DEBUG=jit_dump=<dir>, the generated scene headers and code objects.

Usage: [JIT_PRECISION=f64] jit_report.py [scene[:WxH] ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))


def main():
    import torch
    import rtc_amd
    from rtc_amd import scene_io
    names = sys.argv[1:] or ["three_sphere_scene", "shadow_puppets", "reflect_refract", "refraction", "metal",
                             "cylinders", "cover", "table"]
    for spec in names:
        name, _, size = spec.partition(":")
        w, h = map(int, (size or "1920x1080").split("x"))
        scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
        cam = rtc_amd.camera_resize(scene.camera, w, h)
        with rtc_amd.Context(0) as ctx:
            ctx.set_jit(rtc_amd.RT_JIT_SYNC)
            ctx.upload(scene)
            prec = os.environ.get("JIT_PRECISION", "f32")
            out = torch.empty((h, w, 3), dtype=torch.float32 if prec == "f32" else torch.float64, device="cuda")
            ctx.render_device(cam, out.data_ptr(), 0, 6, prec)
            torch.cuda.synchronize()
            print(name, f"{w}x{h}", prec, ctx.jit_status(), flush=True)


if __name__ == "__main__":
    main()
