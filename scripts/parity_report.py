#!/usr/bin/env python3
"""Parity report: every reference scene rendered on the GPU (f64 and f32
paths) against the f64 oracle.  Writes one JSON object per scene/size with
pixel agreement after 8-bit quantization (canvas.rs:117-123), mean/max |err|
and ray-counter deltas.  The numbers back DESIGN.md's tolerance statement.

Usage: python scripts/parity_report.py [--sizes 160x120,320x240] [--out gpurun_out/parity.json]
       python scripts/parity_report.py --configs   (BASELINE configs[0]-[4] at their own sizes)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

SCENES = ["three_sphere_scene", "reflect_refract", "cover", "table", "cylinders", "metal", "refraction",
          "shadow_puppets"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="160x120,320x240")
    ap.add_argument("--scenes", default=",".join(SCENES))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "parity.json"))
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--configs", action="store_true",
                    help="BASELINE.json configs[0]-[4]: three_sphere 320x240 and 1920x1080, reflect_refract "
                         "1920x1080, cover and table 3840x2160 (each scene at its own size only)")
    args = ap.parse_args()
    import numpy as np

    import pyoracle
    import rtc_amd
    from rtc_amd import scene_io

    rows = []
    ctx = rtc_amd.Context(0)
    if args.configs:
        work = [("three_sphere_scene", ["320x240", "1920x1080"]), ("reflect_refract", ["1920x1080"]),
                ("cover", ["3840x2160"]), ("table", ["3840x2160"])]
    else:
        work = [(name, args.sizes.split(",")) for name in args.scenes.split(",")]
    for name, sizes in work:
        scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
        ctx.upload(scene)
        for size in sizes:
            w, h = map(int, size.split("x"))
            cam = rtc_amd.camera_resize(scene.camera, w, h)
            t0 = time.time()
            ref, rst = pyoracle.render(scene, cam, 6, threads=args.threads)
            t_cpu = time.time() - t0
            qref = pyoracle.quantize(ref).astype(int)
            for prec in ("f64", "f32"):
                img, st = ctx.render(cam, 6, precision=prec)
                img = img.astype(np.float64)
                d8 = np.abs(pyoracle.quantize(img).astype(int) - qref).max(axis=2)
                err = np.abs(img - ref)
                row = {"scene": name, "size": size, "precision": prec,
                       "agree_exact8": float((d8 == 0).mean()), "agree_1lsb": float((d8 <= 1).mean()),
                       "agree_2lsb": float((d8 <= 2).mean()), "mean_abs_err": float(err.mean()),
                       "max_abs_err": float(err.max()),
                       "rays_gpu": int(st["rays"]), "rays_oracle": int(rst["rays"]),
                       "counters_equal": all(st[k] == rst[k] for k in ("primary", "shadow", "reflect", "refract",
                                                                          "shaded")),
                       # per ray kind: (gpu - oracle) / oracle (0 when the oracle has none)
                       "kind_rel_delta": {k: (st[k] - rst[k]) / rst[k] if rst[k] else float(st[k] != 0)
                                          for k in ("primary", "shadow", "reflect", "refract", "shaded")},
                       "kernel_ms": st["kernel_ms"], "oracle_s": t_cpu}
                rows.append(row)
                print(json.dumps(row), flush=True)
    ctx.close()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
