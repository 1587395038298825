#!/usr/bin/env python3
"""GPU probe (not a test): does a hipGraph of K frames shorten a K-frame
region against K separate rt_render_device calls?  configs[1]
(three_sphere at 1920x1080, depth 5, f32), K = 20 (the driver's --steps)
and 1000.  Alternates the two ways ROUNDS times on one context, host clock
around each region (synchronize on both sides, as bench.py), and checks
that a replay renders the same frame and advances the ray counters by K
frames.  Prints one JSON line per way and K.

Usage (GPU box): python scripts/graph_probe.py [rounds]
"""
import json
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", "three_sphere_scene.json"))
    cam = rtc_amd.camera_resize(scene.camera, 1920, 1080)
    torch.cuda.set_device(0)
    ctx = rtc_amd.Context(0)
    ctx.upload(scene)
    img = torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()

    def step(st):
        ctx.render_device(cam, img.data_ptr(), st.cuda_stream, 5, "f32", "real")

    with torch.cuda.stream(s):
        step(s)
        step(s)
        ctx.jit_wait(120000.0)
        for _ in range(2000):
            step(s)
    torch.cuda.synchronize()
    ref = img.clone()
    graphs = {}
    for k in (20, 1000):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(k):
                step(torch.cuda.current_stream())
        graphs[k] = g
    torch.cuda.synchronize()
    img.zero_()
    before = ctx.counters()["rays"]
    graphs[20].replay()
    torch.cuda.synchronize()
    after = ctx.counters()["rays"]
    same = bool(torch.equal(img, ref))
    per_frame = 2 * 1920 * 1080
    res = {("plain", 20): [], ("graph", 20): [], ("plain", 1000): [], ("graph", 1000): []}
    for _ in range(rounds):
        for k in (20, 1000):
            with torch.cuda.stream(s):
                for _ in range(200):  # keep clocks up between regions, as the bench's warm-up does
                    step(s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.cuda.stream(s):
                for _ in range(k):
                    step(s)
            torch.cuda.synchronize()
            res[("plain", k)].append((time.perf_counter() - t0) * 1e3 / k)
            with torch.cuda.stream(s):
                for _ in range(200):
                    step(s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            graphs[k].replay()
            torch.cuda.synchronize()
            res[("graph", k)].append((time.perf_counter() - t0) * 1e3 / k)
    for (way, k), v in res.items():
        print(json.dumps({"way": way, "steps": k, "ms_per_step_median": statistics.median(v),
                          "ms_per_step_min": min(v), "gray_s_median": per_frame / statistics.median(v) / 1e6,
                          "replay_frame_equal": same, "replay_rays": after - before, "expected_rays": 20 * per_frame}))
    ctx.close()


if __name__ == "__main__":
    main()
