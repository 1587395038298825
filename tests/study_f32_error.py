#!/usr/bin/env python3
"""Study (not collected by pytest): where does the f32 path's error against
the f64 oracle come from?  Renders scenes at 320x200 with library builds
that differ only in the f32 math (csrc/rtc_kernels.hip Real<float>) and
reports, per scene, the share of pixels within 2/255 of the oracle after
8-bit quantization, the mean |err| and the ray-count drift.  Frames of 64K
pixels or fewer run the generic kernels (no per-scene build).

Variants are library builds under ray-tracer-challenge-rs_amd/rtc_amd/_lib_<name>/,
made with the Makefile's OUT and EXTRA, e.g.
  make -C ray-tracer-challenge-rs_amd OUT=rtc_amd/_lib_exact EXTRA=-DRTC_F32_EXACT=1 \
       rtc_amd/_lib_exact/librtc.so
  (RTC_F32_EXACT: correctly rounded div/sqrt/pow; RTC_F32_REL_OFFSET=<x>f: the
  over/under-point offset x * max(1, |p|inf))
"default" is the product build (_lib).  The results are in DESIGN.md §4.

Usage: STUDY_VARIANTS="default exact ..." python tests/study_f32_error.py [scene ...]
(on a GPU box)
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIBS = os.path.join(ROOT, "ray-tracer-challenge-rs_amd", "rtc_amd")
VARIANTS = os.environ.get("STUDY_VARIANTS", "default").split()
SCENES = ["refraction", "reflect_refract", "cover", "table", "shadow_puppets"]


def one(variant, scenes):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import pyoracle
    import rtc_amd
    from conftest import scene_fixture
    ctx = rtc_amd.Context(0)
    for name in scenes:
        scene = scene_fixture(name)
        cam = rtc_amd.camera_resize(scene.camera, 320, 200)
        ctx.upload(scene)
        img, st = ctx.render(cam, 6, precision="f32")
        ref, rst = pyoracle.render(scene, cam, 6, threads=16)
        d = np.abs(pyoracle.quantize(img).astype(int) - pyoracle.quantize(ref).astype(int)).max(axis=2)
        print(json.dumps({"variant": variant, "scene": name, "within_2": round(float((d <= 2).mean()), 5),
                          "exact_u8": round(float((d == 0).mean()), 5),
                          "mean_abs": float(np.abs(img.astype(np.float64) - ref).mean()),
                          "rays_rel": (st["rays"] - rst["rays"]) / rst["rays"]}), flush=True)
    ctx.close()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":
        one(sys.argv[2], sys.argv[3:] or SCENES)
        return
    scenes = sys.argv[1:] or SCENES
    for v in VARIANTS:
        lib = os.path.join(LIBS, "_lib" if v == "default" else f"_lib_{v}", "librtc.so")
        env = dict(os.environ, RTC_LIBRARY=lib)
        subprocess.run([sys.executable, __file__, "--variant", v] + scenes, env=env, check=True)


if __name__ == "__main__":
    main()
