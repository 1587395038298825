#!/usr/bin/env python3
"""Diagnostic: kernel time per frame along a camera path (every frame a new
camera: the first launch of each signature), against a repeated camera.

Usage: camera_path.py [scene] [WxH] [frames]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "reflect_refract"
w, h = map(int, (sys.argv[2] if len(sys.argv) > 2 else "1920x1080").split("x"))
n = int(sys.argv[3]) if len(sys.argv) > 3 else 60
scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
base = rtc_amd.camera_resize(scene.camera, w, h)
view = np.linalg.inv(np.array(list(base.inverse)).reshape(4, 4))


def cam_at(k):
    a = float(os.environ.get("PAN", "0.002")) * k  # radians per frame (default ~0.1 degree)
    rot = np.array([[np.cos(a), 0, np.sin(a), 0], [0, 1, 0, 0], [-np.sin(a), 0, np.cos(a), 0], [0, 0, 0, 1.0]])
    return rtc_amd.camera_set_transform(base, rot @ view)


s = torch.cuda.current_stream()
out = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
with rtc_amd.Context(0) as ctx:
    ctx.upload(scene)
    for _ in range(3):
        ctx.render_device(cam_at(0), out.data_ptr(), s.cuda_stream, 6, "f32")
    for label, cams in (("path", [cam_at(k) for k in range(1, n + 1)]), ("repeat", [cam_at(0)] * n)):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        e[0].record(s)
        for c in cams:
            ctx.render_device(c, out.data_ptr(), s.cuda_stream, 6, "f32")
        e[1].record(s)
        torch.cuda.synchronize()
        print(f"{name} {w}x{h} {label}: {e[0].elapsed_time(e[1]) / n:.4f} ms/frame", flush=True)
