#!/usr/bin/env python3
"""Diagnostic: SHA-256 of rendered frames (f32 and f64, every reference scene,
two sizes), to check that two builds produce bit-identical frames:
  RTC_LIBRARY=<build A>/librtc.so python scripts/frame_hashes.py > a.txt
  RTC_LIBRARY=<build B>/librtc.so python scripts/frame_hashes.py > b.txt; diff a.txt b.txt
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

SCENES = ["three_sphere_scene", "shadow_puppets", "reflect_refract", "refraction", "metal", "cylinders", "cover",
          "table"]
with rtc_amd.Context(0) as ctx:
    for name in SCENES:
        scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
        ctx.upload(scene)
        for w, h in ((256, 160), (1920, 1080)):
            cam = rtc_amd.camera_resize(scene.camera, w, h)
            for prec in ("f32", "f64"):
                img, st = ctx.render(cam, 6, precision=prec)
                print(name, f"{w}x{h}", prec, hashlib.sha256(img.tobytes()).hexdigest()[:16], st["rays"], flush=True)
