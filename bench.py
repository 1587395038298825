#!/usr/bin/env python3
"""Benchmark of the MI355X render path — BASELINE.json metric:
"Mray/s (primary+secondary) and ms/frame at 1920x1080, 1/2/4/8 GPU".

A step is one frame: one launch of the persistent tracer over a 1920x1080
canvas of the scene (default scenes/three_sphere_scene.yaml = BASELINE
configs[1]; the YAML's camera with width/height overridden, exactly like
editing the YAML), scene tables and output buffer resident in HBM.  Rays are
counted on the device in the reference's semantics (primary +
shadow + reflect + refract).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py ...):
one process per GPU; frames are independent objects, so each rank renders
its own frame per step with no data-path collective ("scaling": "weak");
value = rays of all ranks / max-over-ranks time.  `--mode tiled` instead
splits ONE frame into cyclic row blocks across ranks and gathers the strips
to rank 0 over RCCL (the north star's tile split; strong scaling).

Prints ONE JSON line on rank 0 with the roofline of the tracer kernel (FP32
compute roof, algorithmic FLOPs of SURVEY.md §8d) and the CPU baseline (the
f64 oracle = C++ restatement of the reference's rayon render_parallel,
timed on this host's cores over a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))
# kernel arguments in device memory (see rtc_amd/__init__.py); before HIP starts
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate
PEAK_FP64_TFLOPS = 78.6   # FP64 vector: vendor spec (the guide lists FP32 only); the f64 parity path
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--scene", default="three_sphere_scene")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--depth", type=int, default=None,
                    help="recursion depth; default 5 for three_sphere_scene (BASELINE configs[1]: 'reflection "
                         "depth 5' — the scene has no reflective or transparent material, so its rays do not "
                         "change) and World::MAX_REFLECTION_ITERATIONS = 6 otherwise")
    ap.add_argument("--precision", choices=["f32", "f64"], default="f32")
    ap.add_argument("--mode", choices=["frames", "tiled"], default="frames")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--flags", type=int, default=0, help="RT_FLAG_* diagnostic ablations (profiling only)")
    return ap.parse_args()


def cpu_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def cpu_baseline(scene, cam, depth, budget_s):
    """f64 oracle render_parallel over this host's cores on whole frames of the
    same workload until `budget_s` elapses (at least one frame)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    threads = cpu_threads()
    rays = frames = 0
    t0 = time.perf_counter()
    while True:
        _, st = pyoracle.render(scene, cam, depth, threads=threads)
        rays += st["rays"]
        frames += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": rays / dt / 1e6, "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"{frames} full {cam.width}x{cam.height} frame(s) of the same scene, depth {depth}, "
                      f"f64 C++ restatement of Camera::render_parallel, {dt:.1f}s on {threads} threads"}


def load_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc pass (profiles/traffic.json)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get(workload)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    if args.depth is None:
        args.depth = 5 if args.scene == "three_sphere_scene" else 6
    import numpy as np
    import torch
    import torch.distributed as dist

    import rtc_amd
    from rtc_amd import dist as rdist
    from rtc_amd import scene_io

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND=gloo and BENCH_SHARE_GPU=1 rehearse the multi-rank
    # path on a one-GPU box (RCCL refuses two ranks on one device); the
    # driver's runs use RCCL ("nccl") with one GPU per rank.
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if os.environ.get("BENCH_SHARE_GPU"):
        local = local % torch.cuda.device_count()
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)

    # Only rank 0 holds the world, as the reference's single caller does; the
    # other ranks receive it (an RCCL broadcast).
    t_first = time.perf_counter()
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{args.scene}.json")) if rank == 0 else None
    if world > 1:
        scene = rdist.broadcast_scene(scene, rank, "cuda" if backend == "nccl" else "cpu")
    cam = rtc_amd.camera_resize(scene.camera, args.width, args.height)
    ctx = rtc_amd.Context(local)
    ctx.upload(scene)
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream
    rdtype = torch.float32 if args.precision == "f32" else torch.float64
    tiled = args.mode == "tiled" and world > 1
    if tiled:
        rows = rdist.strip_height(cam.height, world)
        out = torch.empty((rows, cam.width, 3), dtype=rdtype, device="cuda")
        gathered = torch.empty((world * rows, cam.width, 3), dtype=rdtype, device="cuda") if rank == 0 else None
        image = torch.empty((cam.height, cam.width, 3), dtype=rdtype, device="cuda") if rank == 0 else None
    else:
        out = torch.empty((cam.height, cam.width, 3), dtype=rdtype, device="cuda")
    shard = (rank, world) if tiled else (0, 1)

    def gather():
        rdist.gather_strips(out, gathered, world, rank)
        if rank == 0:
            ctx.assemble_shards(gathered.data_ptr(), cam.width, cam.height, world, 3 * out.element_size(),
                                image.data_ptr(), sptr)

    def step():
        ctx.render_device(cam, out.data_ptr(), sptr, args.depth, args.precision, "real", shard, args.flags)
        if tiled:
            gather()

    step()  # first frame: scene transfer, context, upload and one render
    torch.cuda.synchronize()
    first_frame_ms = (time.perf_counter() - t_first) * 1e3
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    before = ctx.counters()

    # Device time of the tracer launches, from HIP events on the launch stream.
    # Frames mode: ONE event pair brackets the K back-to-back launches (per-launch
    # event records cost ~6 us of GPU time per frame on MI355X — they stop the
    # next launch's waves from overlapping the previous one's tail — see
    # scripts/host_overhead.py), so the average launch duration is the bracket
    # / K.  Tiled mode: a pair around each render call, excluding the gather.
    n_ev = args.steps if tiled else 1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_ev)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if tiled:
        for i in range(args.steps):
            ev[i][0].record(stream)
            ctx.render_device(cam, out.data_ptr(), sptr, args.depth, args.precision, "real", shard, args.flags)
            ev[i][1].record(stream)
            gather()
    else:
        ev[0][0].record(stream)
        for _ in range(args.steps):
            step()
        ev[0][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    after = ctx.counters()
    launch_ms = float(np.sum([a.elapsed_time(b) for a, b in ev])) / args.steps

    rays = after["rays"] - before["rays"]
    flops = after["algorithmic_flops"] - before["algorithmic_flops"]
    elapsed, total_rays = rdist.job_totals(elapsed, rays, "cuda" if backend == "nccl" else "cpu")
    if rank == 0:
        flops_per_launch = flops / args.steps
        peak = PEAK_FP32_TFLOPS if args.precision == "f32" else PEAK_FP64_TFLOPS
        achieved = flops_per_launch / (launch_ms * 1e-3) / 1e12
        workload = f"{args.scene}@{cam.width}x{cam.height},depth={args.depth},{args.precision}"
        traffic = load_traffic(workload)
        line = {
            "metric": "Mray/s (primary+secondary) and ms/frame at 1920x1080",
            "value": total_rays / elapsed / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if tiled else "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic: the reference's scene (scenes/%s.yaml) rendered at the configured size" % args.scene,
            "config": {"workload": workload, "scene": args.scene, "width": cam.width, "height": cam.height,
                       "max_depth": args.depth, "parallelism": f"{'tiles' if tiled else 'frames'}x{world}",
                       "rays_per_frame": int(rays // args.steps), "mode": args.mode},
            "roofline": {"bound": "mfma", "pipe": f"valu-{args.precision}", "achieved": achieved, "peak": peak,
                         "unit": "TFLOP/s", "frac": achieved / peak, "traffic": traffic,
                         "kernel_ms": launch_ms, "flops_per_launch": flops_per_launch,
                         # the north star's HBM view: PMC bytes per launch over the launch time,
                         # against the ~8 TB/s memory roof (a diagnostic: the path is compute-bound)
                         "hbm_gbs": traffic / (launch_ms * 1e-3) / 1e9 if traffic else None,
                         "hbm_frac": traffic / (launch_ms * 1e-3) / 1e9 / PEAK_HBM_GBS if traffic else None},
        }
        line["first_frame_ms"] = first_frame_ms
        if not tiled:
            # a drop-in Camera::render: synchronous rt_render into host memory,
            # PCIe copy included (median of 10; never `value`)
            lat = []
            for _ in range(10):
                t = time.perf_counter()
                ctx.render(cam, args.depth, args.precision)
                lat.append((time.perf_counter() - t) * 1e3)
            line["host_frame_ms"] = float(np.median(lat))
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene, cam, args.depth, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
