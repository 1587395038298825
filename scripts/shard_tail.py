"""Diagnostic: where one shard of a multi-GPU frame spends its
time.  For each listed shard of an N-way split: the event-timed frame, the
per-workgroup stamps (start/end quantiles), the recorded tile costs (mean
workgroup load, heaviest tiles and what their parts cost), all on the per-scene
kernels as a warm renderer runs them.
Usage: python scripts/shard_tail.py [scene W H N shard,shard,...]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cover"
w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (3840, 2160)
n = int(sys.argv[4]) if len(sys.argv) > 4 else 8
which = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [0]
scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json"))
cam = rtc_amd.camera_resize(scene.camera, w, h)
s = torch.cuda.current_stream()
q = lambda a: [round(float(np.quantile(a, p)), 1) for p in (0, 0.1, 0.5, 0.9, 0.99, 1.0)]  # noqa: E731
with rtc_amd.Context(0) as ctx:
    ctx.set_jit(rtc_amd.RT_JIT_SYNC)
    ctx.upload(scene)
    rows = rtc_amd.shard_rows(h, n)
    out = torch.empty((rows, w, 3), dtype=torch.uint8, device="cuda")
    for k in which:
        for _ in range(12):
            ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, n))
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, n))
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        cost = ctx.debug_tile_costs().astype(np.float64) * 1e-2  # us (10 ns ticks)
        ctx.render_device(cam, out.data_ptr(), s.cuda_stream, 6, "f32", "u8", (k, n), rtc_amd.RT_FLAG_STAMPS)
        torch.cuda.synchronize()
        st = ctx.debug_stamps().astype(np.int64)
        t0 = st[:, 0].min()
        start, end = (st[:, 0] - t0) * 1e-2, (st[:, 1] - t0) * 1e-2
        grid = len(st)
        live = cost[cost > 0]
        mean_load = live.sum() / grid
        top = np.sort(live)[::-1][:12]
        res = {"scene": name, "size": f"{w}x{h}", "shard": f"{k}/{n}", "event_ms_median": round(float(np.median(ts)), 4),
               "grid": grid, "tiles": int(len(live)), "sum_cost_us": round(float(live.sum()), 1),
               "mean_wg_load_us": round(float(mean_load), 1), "top_tile_cost_us": [round(float(x), 1) for x in top],
               "top_over_mean": round(float(top[0] / mean_load), 2),
               "stamp_span_us": round(float(end.max()), 1), "start_q_us": q(start), "end_q_us": q(end),
               "dur_q_us": q(end - start),
               "wg_busy_frac": round(float((end - start).sum() / (grid * end.max())), 3)}
        # how many workgroups are still running at each time: the tail's width
        grid_t = np.linspace(0, end.max(), 21)
        res["running_at_5pct_steps"] = [int(((start <= t) & (end > t)).sum()) for t in grid_t]
        log = ctx.debug_item_log().astype(np.int64)
        if len(log):
            item, wg = log[:, 0] & 0xFFFFFFFF, log[:, 0] >> 32
            s0, e0 = (log[:, 1] - t0) * 1e-2, (log[:, 2] - t0) * 1e-2
            dur = e0 - s0
            split, prio = (item >> 24) & 7, (item >> 27) & 3
            last = np.argsort(e0)[::-1][:12]
            res["items"] = int(len(log))
            res["item_dur_q_us"] = q(dur)
            res["items_by_split"] = np.bincount(split, minlength=4).tolist()
            res["items_by_prio"] = np.bincount(prio, minlength=4).tolist()
            res["last_items"] = [{"start": round(float(s0[i]), 1), "dur": round(float(dur[i]), 1), "split": int(split[i]),
                                  "prio": int(prio[i]), "wg_items": int((wg == wg[i]).sum())} for i in last]
            longest = np.argsort(dur)[::-1][:8]
            res["longest_items"] = [{"start": round(float(s0[i]), 1), "dur": round(float(dur[i]), 1), "split": int(split[i]),
                                     "prio": int(prio[i])} for i in longest]
            late = s0 > 0.5 * end.max()
            res["items_started_after_half_span"] = int(late.sum())
            res["late_item_dur_q_us"] = q(dur[late]) if late.any() else None
        print(json.dumps(res), flush=True)
