#!/usr/bin/env python3
"""GPU probe (not a test): the driver's short region (K = 20 frames) with two
frames in flight, as bench.py times it, against variants without parts of
it.  configs[1] (three_sphere 1920x1080, depth 5, f32), two contexts on two
side streams with the frames-in-flight hint.  Each round: 200 untimed
frames, a re-warm burst, synchronize, then the variant, host clock between
synchronizes:
  bench     counters read (device sync + copy per context), t0, event +
            cross-stream wait, K frames, joins + event, sync (bench.py)
  nocount   bench without the counters read before t0
  nojoin    t0, K frames, sync (no events, no cross-stream waits)
  spin      nojoin with the host polling each stream's last event before the sync
Median and min us per frame over ROUNDS rounds, plus the 1000-frame rate and
the host's own submission time per frame within it.
Usage (GPU box): python scripts/region_inflight_probe.py [rounds]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def main():
    import torch

    import rtc_amd
    from rtc_amd import scene_io
    from bench import timed_launches
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    k = 20
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", "three_sphere_scene.json"))
    cam = rtc_amd.camera_resize(scene.camera, 1920, 1080)
    ctxs = [rtc_amd.Context(0) for _ in range(2)]
    for c in ctxs:
        c.upload(scene)
        c.set_frames_in_flight(2)
    imgs = [torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda") for _ in ctxs]
    streams = [torch.cuda.Stream() for _ in ctxs]
    turn = [0]

    def step():
        i = turn[0]
        turn[0] = 1 - i
        ctxs[i].render_device(cam, imgs[i].data_ptr(), streams[i].cuda_stream, 5, "f32", "real")

    for _ in range(4):
        step()
    for c in ctxs:
        c.jit_wait(120000.0)
    timed = timed_launches(step, streams, k)
    for _ in range(2000):
        step()
    torch.cuda.synchronize()

    def region(variant):
        for _ in range(200):
            step()
        torch.cuda.synchronize()
        for _ in range(170):  # bench.py's re-warm burst (~2 ms of frames)
            step()
        torch.cuda.synchronize()
        turn[0] = 0
        if variant == "bench":
            for c in ctxs:
                c.counters()
        t0 = time.perf_counter()
        if variant == "nojoin":
            for _ in range(k):
                step()
            torch.cuda.synchronize()
        elif variant == "spin":  # nojoin, but the host polls the streams' last events before synchronizing
            for _ in range(k):
                step()
            for e, st in zip(ends, streams):
                e.record(st)
            while not all(e.query() for e in ends):
                pass
            torch.cuda.synchronize()
        else:
            timed()
        return (time.perf_counter() - t0) * 1e6 / k

    ends = [torch.cuda.Event() for _ in streams]
    for e, st in zip(ends, streams):
        e.record(st)
    res = {v: [] for v in ("bench", "nocount", "nojoin", "spin")}
    for _ in range(rounds):
        for v in res:
            res[v].append(region(v))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(1000):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    steady = (time.perf_counter() - t0) * 1e6 / 1000
    host_submit = (t1 - t0) * 1e6 / 1000  # the host's own time per step (no wait on the GPU)
    out = {v: {"median_us": round(statistics.median(x), 2), "min_us": round(min(x), 2)} for v, x in res.items()}
    out["steady_1000_us"] = round(steady, 2)
    out["host_submit_us"] = round(host_submit, 2)
    print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
