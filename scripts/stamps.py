#!/usr/bin/env python3
"""Diagnostic: per-workgroup start/end timestamps (RT_FLAG_STAMPS) of one
frame, summarised: kernel span, dispatch ramp, workgroup duration quantiles,
tail.  Ticks are s_memrealtime (100 MHz = 10 ns).

Usage: python scripts/stamps.py [--scene S] [--flags F] [--sched grid|static|dynamic]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="three_sphere_scene")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--precision", default="f32")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--out", default="real", choices=["real", "u8"])
    ap.add_argument("--shard", default="0/1", help="shard_index/shard_count")
    args = ap.parse_args()
    import numpy as np
    import torch

    import rtc_amd
    from rtc_amd import scene_io

    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{args.scene}.json"))
    cam = rtc_amd.camera_resize(scene.camera, args.width, args.height)
    ctx = rtc_amd.Context(0)
    ctx.upload(scene)
    dt = torch.uint8 if args.out == "u8" else (torch.float32 if args.precision == "f32" else torch.float64)
    si, sn = map(int, args.shard.split("/"))
    rows = rtc_amd.shard_rows(cam.height, sn)
    out = torch.empty((rows, cam.width, 3), dtype=dt, device="cuda")
    for _ in range(5):
        ctx.render_device(cam, out.data_ptr(), 0, 6, args.precision, args.out, (si, sn), args.flags | 8)
    torch.cuda.synchronize()
    st = ctx.debug_stamps().astype(np.int64)
    t0 = st[:, 0].min()
    start = (st[:, 0] - t0) * 10e-3  # us
    end = (st[:, 1] - t0) * 10e-3
    dur = end - start
    q = lambda a: [round(float(np.quantile(a, p)), 2) for p in (0, 0.1, 0.5, 0.9, 1.0)]  # noqa: E731
    # kernel-only time of the same launch without stamps, by events
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(50):
        ctx.render_device(cam, out.data_ptr(), 0, 6, args.precision, args.out, (si, sn), args.flags)
    ev[1].record()
    torch.cuda.synchronize()
    res = {"label": f"{args.scene} flags={args.flags} out={args.out} sched={os.environ.get('RTC_DEBUG', 'default')}",
           "launch_us": round(ev[0].elapsed_time(ev[1]) * 1e3 / 50, 2),
           "workgroups": int(len(st)), "span_us": round(float(end.max()), 2),
           "start_q_us": q(start), "dur_q_us": q(dur), "end_q_us": q(end)}
    if os.environ.get("STAMPS_DETAIL"):
        late = np.where(start > 5.0)[0]
        res["late_starters"] = int(len(late))
        res["late_by_queue"] = np.bincount(late % 8, minlength=8).tolist()
        res["end_max_by_queue_us"] = [round(float(end[np.arange(len(end)) % 8 == q].max()), 1) for q in range(8)]
        res["end_med_by_queue_us"] = [round(float(np.median(end[np.arange(len(end)) % 8 == q])), 1) for q in range(8)]
    print(json.dumps(res))
    ctx.close()


if __name__ == "__main__":
    main()
