#!/usr/bin/env python3
"""Benchmark of the MI355X render path — BASELINE.json metric:
"Mray/s (primary+secondary) and ms/frame at 1920x1080, 1/2/4/8 GPU".

A step is one frame, scene tables and output buffer resident in HBM.  Rays
are counted on the device in the reference's semantics (SURVEY.md §8d:
primary + shadow + reflect + refract).

* A step renders configs[1] on every GPU: one launch of the persistent
  tracer over a 1920x1080 canvas of scenes/three_sphere_scene.yaml (the
  YAML's camera with width/height overridden, exactly like editing the
  YAML), f32 framebuffer.  With N GPUs (python -m torch.distributed.run
  --nproc-per-node N bench.py --gpus N ...; one process per GPU) each GPU
  renders its own frame per step (independent frames: no data-path
  collective, "scaling": "weak"), so the line's workload per GPU is the same
  at every N and `value` is the whole job's rays / time.
* The default run then also measures the north star's image-tile split, at
  every N (N = 1 included): BASELINE configs[3] and configs[4],
  scenes/cover.yaml and scenes/table.yaml at 3840x2160, every frame
  split across the N GPUs in cyclic row blocks by librtc's own multi-GPU
  context (csrc/rtc_group.cpp: the scene RCCL-broadcast by rt_scene_upload,
  the strips RCCL-gathered onto rank 0 and de-interleaved there), gathering
  the 8-bit canvas (canvas.rs:117-123; 4x fewer bytes than f32), and attaches
  them as "tile_split": {"cover": ..., "table": ...}, each with its Mray/s and ms/frame, per-shard render / gather /
  end-to-end milliseconds, and the same frame on rank 0's GPU alone
  (`single_gpu_ms_per_step`, `speedup_vs_1gpu`).  `--mode tiled` makes the
  split the line itself ("scaling": "strong"); `--mode frames` skips it.

Prints ONE JSON line on rank 0 with the roofline of the tracer kernel (FP32
VALU roof, algorithmic FLOPs of SURVEY.md §8d) and, on one GPU, the CPU
baseline (the f64 oracle = C++ restatement of the reference's rayon
render_parallel, timed on this host's cores over a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
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
    ap.add_argument("--warmup-ms", type=float, default=200.0,
                    help="keep warming up (untimed) until at least this much wall time of frames has run, "
                         "whatever --warmup: a few 25 us frames leave the GPU below its steady clocks")
    ap.add_argument("--mode", choices=["auto", "frames", "tiled"], default="auto",
                    help="auto: a frame per GPU per step, plus the configs[3]/[4] tile splits as 'tile_split'; "
                         "frames: without it; tiled: the tile split is the line")
    ap.add_argument("--scene", default=None,
                    help="default three_sphere_scene (configs[1]) on one GPU / in frames mode, cover (configs[3]) "
                         "when tiled")
    ap.add_argument("--width", type=int, default=None, help="default 1920 (3840 for the tiled default)")
    ap.add_argument("--height", type=int, default=None, help="default 1080 (2160 for the tiled default)")
    ap.add_argument("--depth", type=int, default=None,
                    help="recursion depth; default 5 for three_sphere_scene (BASELINE configs[1]: 'reflection "
                         "depth 5' — the scene has no reflective or transparent material, so its rays do not "
                         "change) and World::MAX_REFLECTION_ITERATIONS = 6 otherwise")
    ap.add_argument("--precision", choices=["f32", "f64"], default="f32")
    ap.add_argument("--out", choices=["real", "u8"], default=None,
                    help="framebuffer format: default real (f32) on one GPU, u8 (the quantized canvas) when tiled")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--flags", type=int, default=0, help="RT_FLAG_* diagnostic ablations (profiling only)")
    ap.add_argument("--gather", choices=["rccl", "peer"], default="rccl",
                    help="tiled: how rank 0 gets the shards (rtc.h rt_context_set_gather); the other mode is "
                         "measured too and reported under gather_variants")
    ap.add_argument("--ab", action="store_true",
                    help="A/B runs: skip the one-shot child, the host-frame latency and the per-generation frame")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight: consecutive steps alternate between this many contexts, each on a "
                         "stream of its own, so one frame's launch tail overlaps the next frame's start (1 = "
                         "every frame on one stream, one after another); default 3 for frames, 2 when tiled "
                         "(each a group context with its own RCCL communicator)")
    ap.add_argument("--stream", choices=["side", "null"], default="side",
                    help="the launch stream: a stream of the bench's own (default) or HIP's null stream")
    ap.add_argument("--one-shot-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def cpu_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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
    return {"value": rays / dt / 1e6, "unit": "Mray/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
            "sample": f"{frames} full {cam.width}x{cam.height} frame(s) of the same scene, depth {depth}, "
                      f"f64 C++ restatement of Camera::render_parallel, {dt:.1f}s on {threads} threads"}


def cpu_serial_configs0(budget_s):
    """BASELINE configs[0]: three_sphere_scene at 320x240 in serial CPU mode,
    i.e. the f64 oracle's restatement of Camera::render (camera.rs:79-95) on
    one thread, whole frames until `budget_s` elapses (at least 3)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    import rtc_amd
    from rtc_amd import scene_io
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", "three_sphere_scene.json"))
    cam = rtc_amd.camera_resize(scene.camera, 320, 240)
    times, rays = [], 0
    t0 = time.perf_counter()
    while len(times) < 3 or time.perf_counter() - t0 < budget_s:
        t = time.perf_counter()
        _, st = pyoracle.render(scene, cam, 6, threads=1)
        times.append(time.perf_counter() - t)
        rays += st["rays"]
    ms = statistics.median(times) * 1e3
    return {"config": "scenes/three_sphere_scene.yaml at 320x240, serial CPU mode (BASELINE configs[0])",
            "ms_per_frame": ms, "value": rays / sum(times) / 1e6, "unit": "Mray/s", "cores": 1,
            "kind": "port", "rays_per_frame": st["rays"],
            "sample": f"{len(times)} frames, f64 C++ restatement of Camera::render on 1 thread, median ms/frame"}


def load_profile(name: str, workload: str):
    """Per-workload figures from the committed rocprofv3 --pmc passes
    (scripts/collect_profiles.py): profiles/traffic.json (HBM bytes per
    launch), profiles/issue.json (VALU issue and wait fractions)."""
    p = os.path.join(ROOT, "profiles", name)
    try:
        with open(p) as f:
            return json.load(f).get(workload)
    except (OSError, ValueError):
        return None


_SMI = {}


def device_state(local: int) -> dict:
    """The GPU's clocks, power and temperature from amdsmi (read-only; no
    HIP call), so a bench line taken on a slow box can be told from a slow
    build: current gfx and memory clocks (MHz), socket power and its cap (W),
    hotspot temperature (C), and the throttle status when the metrics table
    has one.  {"error": ...} when amdsmi is unavailable (never fails the line)."""
    if os.environ.get("BENCH_NO_SMI"):
        return {"skipped": "BENCH_NO_SMI"}
    try:
        import amdsmi
        if "handle" not in _SMI:
            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            pick = None
            try:  # this rank's device by PCI bus id (amdsmi lists every GPU of the node)
                import torch
                p = torch.cuda.get_device_properties(local)
                want = (getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None))
                for h in handles:
                    bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
                    bus, dev = int(bdf.split(":")[1], 16), int(bdf.split(":")[2].split(".")[0], 16)
                    if want[0] is not None and (bus, dev) == want:
                        pick = h
            except Exception:  # noqa: BLE001
                pick = None
            if pick is None and len(handles) == 1:
                pick = handles[0]
            if pick is None:
                return {"error": f"amdsmi: {len(handles)} GPUs, none matched cuda:{local}"}
            _SMI["handle"] = pick
            _SMI["bdf"] = amdsmi.amdsmi_get_gpu_device_bdf(pick)
        h = _SMI["handle"]
        out = {"bdf": _SMI["bdf"], "t": time.time()}

        def get(key, fn):
            try:
                out[key] = fn()
            except Exception as e:  # noqa: BLE001  (one missing field does not lose the rest)
                out[key] = None
                out.setdefault("missing", []).append(f"{key}: {type(e).__name__}")
        get("sclk_mhz", lambda: amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)["clk"])
        get("mclk_mhz", lambda: amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.MEM)["clk"])
        get("power_w", lambda: _power(amdsmi.amdsmi_get_power_info(h)))
        get("power_cap_w", lambda: amdsmi.amdsmi_get_power_cap_info(h)["power_cap"] / 1e6)
        get("hotspot_c", lambda: amdsmi.amdsmi_get_temp_metric(h, amdsmi.AmdSmiTemperatureType.HOTSPOT,
                                                               amdsmi.AmdSmiTemperatureMetric.CURRENT))
        get("power_cap_raw", lambda: amdsmi.amdsmi_get_power_cap_info(h)["power_cap"])

        def metrics():
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            return {k: m.get(k) for k in ("current_gfxclk", "average_gfxclk_frequency", "current_uclk",
                                          "temperature_hotspot", "average_socket_power", "throttle_status")}
        get("metrics", metrics)
        return out
    except Exception as e:  # noqa: BLE001  (a diagnostic: never fails the bench line)
        return {"error": repr(e)[:200]}


def _power(info: dict):
    for k in ("current_socket_power", "socket_power", "average_socket_power"):
        v = info.get(k)
        if isinstance(v, (int, float)) and v not in (0, 0xFFFF, 0xFFFFFFFF):
            return v
    return None


def timed_launches(fn, stream, n):
    """Device milliseconds of n back-to-back calls of fn(), one event pair on
    `stream` (a list: the first stream opens the bracket, the others join its
    start and are joined back before it closes).  The events are created
    (torch makes the HIP event at its first record) and recorded once before
    the caller's clock starts: a lazy hipEventCreate inside a 20-frame region
    added ~70 us to it (scripts/short_region_probe.py)."""
    import torch
    streams = stream if isinstance(stream, (list, tuple)) else [stream]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    joins = [torch.cuda.Event() for _ in streams[1:]]
    e0.record(streams[0])
    e1.record(streams[0])
    for j, s in zip(joins, streams[1:]):
        j.record(s)
    torch.cuda.synchronize()

    def run():
        e0.record(streams[0])
        for s in streams[1:]:
            s.wait_event(e0)
        for _ in range(n):
            fn()
        for j, s in zip(joins, streams[1:]):
            j.record(s)
            streams[0].wait_event(j)
        e1.record(streams[0])
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)
    return run


def resolve(args, tiled):
    """Fill the workload defaults: configs[1] (three_sphere at 1920x1080, f32
    frames) unless tiled, configs[3] (cover at 3840x2160, u8 canvas) when tiled."""
    a = argparse.Namespace(**vars(args))
    if a.scene is None:
        a.scene = "cover" if tiled else "three_sphere_scene"
    default_4k = tiled and a.scene in SPLIT_SCENES
    a.width = a.width or (3840 if default_4k else 1920)
    a.height = a.height or (2160 if default_4k else 1080)
    a.out = a.out or ("u8" if tiled else "real")
    if a.depth is None:
        a.depth = 5 if a.scene == "three_sphere_scene" else 6
    return a


def one_shot_child(args):
    """A drop-in one-shot render in a fresh, torch-free process (what the
    reference's only caller does, main.rs:13-22: load, then time one
    render call; a Rust host would bind librtc the same way): context
    creation (the HIP runtime starts here), scene upload, then one
    synchronous rt_render into a host canvas (the cold generic kernel, module
    load and PCIe copy included).  Prints one JSON object."""
    os.environ["RTC_NO_TORCH"] = "1"
    # the CLI's setting (rtc_cli.cpp main): frame copies as blit
    # kernels, not on an SDMA engine whose first use costs 8-12 ms
    os.environ.setdefault("GPU_FORCE_BLIT_COPY_SIZE", "1048576")
    import numpy as np
    import rtc_amd
    from rtc_amd import scene_io
    a = resolve(args, False)
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{a.scene}.json"))
    cam = rtc_amd.camera_resize(scene.camera, a.width, a.height)
    canvas = np.zeros((cam.height, cam.width, 3), dtype=np.float32 if a.precision == "f32" else np.float64)
    t0 = time.perf_counter()
    ctx = rtc_amd.Context(0)
    t1 = time.perf_counter()
    ctx.upload(scene)
    t2 = time.perf_counter()
    _, st = ctx.render(cam, a.depth, a.precision, "real", out=canvas)
    t3 = time.perf_counter()
    ctx.set_jit(rtc_amd.RT_JIT_OFF)  # (no per-scene build from a one-shot process)
    _, st2 = ctx.render(cam, a.depth, a.precision, "real", out=canvas)  # the same call, warm
    t4 = time.perf_counter()
    print(json.dumps({"context_ms": (t1 - t0) * 1e3, "upload_ms": (t2 - t1) * 1e3, "render_ms": (t3 - t2) * 1e3,
                      "total_ms": (t3 - t0) * 1e3, "render_kernel_ms": st["kernel_ms"],
                      "second_render_ms": (t4 - t3) * 1e3, "jit_used": ctx.jit_status()["used"],
                      "workload": f"{a.scene}@{cam.width}x{cam.height},depth={a.depth},{a.precision}"}))
    ctx.close()


def one_shot(args, env=None, runs=3):
    """Run one_shot_child in `runs` fresh subprocesses (rank 0, N = 1) and
    report the median of each timing (a single start-up sample varies by
    2x between runs); {"error": ...} if a run fails.  `env`: extra
    environment of the child (the SDMA-copy variant)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--one-shot-child", "--precision", args.precision]
    for k in ("scene", "width", "height", "depth"):
        if getattr(args, k) is not None:
            cmd += [f"--{k}", str(getattr(args, k))]
    samples = []
    try:
        for _ in range(runs):
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env={**os.environ, **(env or {})})
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not lines:
                return {"error": (r.stderr or r.stdout)[-400:]}
            samples.append(json.loads(lines[-1]))
    except Exception as e:  # noqa: BLE001  (a diagnostic: never fails the bench line)
        return {"error": repr(e)[:400]}
    out = dict(samples[0])
    for k, v in samples[0].items():
        if isinstance(v, float):
            out[k] = float(statistics.median(s[k] for s in samples))
    out["runs"] = runs
    out["total_ms_samples"] = [round(s["total_ms"], 2) for s in samples]
    return out


def main():
    args = parse()
    if args.one_shot_child:
        one_shot_child(args)
        return
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_SHARE_GPU=1 rehearses several ranks on a one-GPU box (frames mode;
    # RCCL refuses two ranks on one device, so the tiled group needs one GPU each)
    if os.environ.get("BENCH_SHARE_GPU"):
        local = local % torch.cuda.device_count()
    # control plane (ids, camera, barriers, max-over-ranks): gloo on the host;
    # the data path's collectives are librtc's own RCCL calls
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    # The line's workload is the same at every N (the driver divides the
    # N-GPU value by N x the 1-GPU value): configs[1], one frame per GPU per
    # step, "weak" (--mode auto|frames).  With N > 1 the auto mode then also
    # measures the north star's image-tile split of configs[3] (cover at 4K
    # split across the N GPUs by librtc's RCCL group) and attaches it as
    # "tile_split"; --mode tiled makes that split the line itself.
    tiled = args.mode == "tiled"
    # the device state before anything runs (measure: why not next to the region)
    state0 = device_state(local)
    line = measure(resolve(args, tiled), tiled, world, rank, local, state0)
    if args.mode == "auto":
        # The north star's strong-scaling series, at every N (N = 1 included,
        # so a scaling curve compares one workload): configs[3] and configs[4],
        # each 4K frame split across the N GPUs by librtc's group context.
        splits = {}
        for name in SPLIT_SCENES:
            split = measure(resolve(args_for_split(args, name), True), True, world, rank, local)
            if rank == 0:
                splits[name] = {k: split[k] for k in (
                    "value", "unit", "ms_per_step", "steps", "scaling", "config", "render_ms_per_shard",
                    "gather_ms", "frame_ms", "gather", "gather_variants", "single_gpu_ms_per_step",
                    "speedup_vs_1gpu", "strong_scaling_efficiency", "single_gpu_value", "roofline",
                    "first_frame_ms", "device_state", "shards_of_8_on_one_gpu") if k in split}
        if rank == 0:
            line["scaling_note"] = (
                "value: N independent configs[1] frames per step, one per GPU (weak scaling: a throughput check, "
                "linear by construction) - NOT a scaling result. The north star's image-tile split is tile_split: "
                "configs[3] (cover) and configs[4] (table) at 3840x2160, each frame split across the N GPUs "
                "(strong scaling: speedup_vs_1gpu over the same frame on one GPU, at every N)")
            line["tile_split"] = splits
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# BASELINE configs[3] and configs[4]: the 4K frames the north star splits across GPUs
SPLIT_SCENES = ("cover", "table")


def args_for_split(args, scene):
    """The tile-split series' workload (configs[3] / configs[4] at 3840x2160,
    u8 canvas); the line's own --scene/--width/--height/--out/--depth describe
    its frames."""
    a = argparse.Namespace(**vars(args))
    a.scene = scene
    a.width = a.height = a.out = a.depth = None
    return a


def measure(args, tiled, world, rank, local, state_before=None):
    """One workload on this rank's GPU (frames) or split across the group
    (tiled); returns rank 0's JSON line (None elsewhere)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import rtc_amd
    from rtc_amd import dist as rdist
    from rtc_amd import scene_io
    # The device state before anything of this workload runs: an amdsmi query
    # next to the timed region slowed its frames by 20 % (round 6, same box,
    # three_sphere 1080p: 15.7 -> 18.8 us per frame with a sample right
    # before the region), so the samples are taken before the
    # context, the first frame and the >= 200 ms warm-up, and after the
    # region's clock has stopped.
    if state_before is None:
        state_before = device_state(local)
    # Only rank 0 holds the world, as the reference's single caller does
    t_first = time.perf_counter()
    scene = scene_io.load(os.path.join(ROOT, "tests", "golden", "scenes", f"{args.scene}.json")) if rank == 0 else None
    phase = {"scene_load_ms": (time.perf_counter() - t_first) * 1e3}
    # the frames run on a stream of their own (HIP's null stream orders every
    # launch against the device's other blocking streams; --stream null keeps
    # it for the A/B)
    # Frames in flight (--inflight F): consecutive steps alternate between F
    # contexts, each with its own stream and output buffer, so a frame's
    # launch tail (its last workgroups) overlaps the next frame's first
    # ones.  Round 6, same box (scripts/overlap_probe.py): three_sphere 1080p
    # 15.65 -> 12.59 us per frame, a cover 4K shard of 8 0.125 -> 0.103 ms,
    # table's 0.141 -> 0.114, reflect_refract 0.236 -> 0.220; frames equal.
    # Each frame is whole and independent (a context renders it from its own
    # resident scene copy), as a renderer producing an animation would run.
    # Default 3 for frames: same box, the driver's flags, eight alternating
    # rounds, 3 ahead of 2 in every one (mean 308.5 against 293.5 Gray/s;
    # 4: 253-274), equal at 1000 frames (profiles/ab/r06_inflight_3.txt).
    # Tiled lines keep 2 (equal at N = 1, one communicator per frame in flight).
    inflight = max(1, args.inflight if args.inflight else (2 if tiled else 3))
    # the frames run on streams of their own (HIP's null stream orders every
    # launch against the device's other blocking streams; --stream null keeps
    # it for the A/B, with one frame in flight)
    if args.stream == "null":
        inflight = 1
    streams = [torch.cuda.Stream() if args.stream == "side" else torch.cuda.current_stream() for _ in range(inflight)]
    stream = streams[0]
    sptr = stream.cuda_stream
    rdtype = torch.uint8 if args.out == "u8" else (torch.float32 if args.precision == "f32" else torch.float64)
    if tiled:
        # the library's multi-GPU context: RCCL communicator from a unique id,
        # scene broadcast inside rt_scene_upload, strips gathered onto rank 0
        # (one group per frame in flight: each its own communicator)
        uids = [rdist.share_unique_id(rank) if world > 1 else rtc_amd.comm_unique_id() for _ in range(inflight)]
        t = time.perf_counter()
        ctxs = [rtc_amd.Context.rank(local, world, rank, u) for u in uids]
        for c in ctxs:
            c.set_gather(rtc_amd.RT_GATHER_PEER if args.gather == "peer" else rtc_amd.RT_GATHER_RCCL)
        phase["context_ms"] = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        # every rank raises if any rank's part of the upload failed (no rank
        # left waiting in the next collective: rdist.collective_call)
        for c in ctxs:
            rdist.collective_call(lambda: c.upload(scene if rank == 0 else None), rank)
        phase["upload_ms"] = (time.perf_counter() - t) * 1e3
        cam0 = rtc_amd.camera_resize(scene.camera, args.width, args.height) if rank == 0 else None
        cam = rdist.share_camera(cam0, rank) if world > 1 else cam0
        images = [torch.empty((cam.height, cam.width, 3), dtype=rdtype, device="cuda") if rank == 0 else None
                  for _ in range(inflight)]
    else:
        if world > 1:
            scene = rdist.broadcast_scene(scene, rank, "cpu")
        cam = rtc_amd.camera_resize(scene.camera, args.width, args.height)
        t = time.perf_counter()
        ctxs = [rtc_amd.Context(local) for _ in range(inflight)]
        phase["context_ms"] = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        for c in ctxs:
            c.upload(scene)
        phase["upload_ms"] = (time.perf_counter() - t) * 1e3
        images = [torch.empty((cam.height, cam.width, 3), dtype=rdtype, device="cuda") for _ in range(inflight)]
    if inflight > 1:  # (rtc.h planning hint: the direct kernel's grid for throughput)
        for c in ctxs:
            c.set_frames_in_flight(inflight)
    ctx, image = ctxs[0], images[0]
    out_ptrs = [im.data_ptr() if im is not None else None for im in images]
    sptrs = [s_.cuda_stream for s_ in streams]
    turn = [0]

    def step_on(i):
        ctxs[i].render_device(cam, out_ptrs[i], sptrs[i], args.depth, args.precision, args.out, (0, 1), args.flags)

    def step():  # the next frame, round robin over the frames in flight
        i = turn[0]
        turn[0] = (i + 1) % inflight
        step_on(i)

    def step0():  # one frame on the first context (latency, cold launches)
        step_on(0)

    def counters_sum():
        cs = [c.counters() for c in ctxs]
        return {k: sum(c_[k] for c_ in cs) for k in ("rays", "algorithmic_flops", "primary", "shadow", "reflect",
                                                      "refract")}

    t = time.perf_counter()
    step0()  # first frame: scene transfer, context, upload and one render
    torch.cuda.synchronize()
    phase["first_render_ms"] = (time.perf_counter() - t) * 1e3
    first_frame_ms = (time.perf_counter() - t_first) * 1e3
    if rank == 0:  # the frame into host memory (the rest of a one-shot Camera::render)
        t = time.perf_counter()
        image.cpu()
        phase["d2h_ms"] = (time.perf_counter() - t) * 1e3
    # The per-scene kernel (rtc.h RT_JIT_AUTO): the second large frame starts
    # its hipRTC build on a host thread and renders with the generic kernel;
    # frames switch once it lands.  The bench lets it land before the warm-up
    # so the timed region measures the steady-state kernel (untimed, reported).
    t_j = time.perf_counter()
    step0()
    jit_pending = ctx.jit_wait(120000.0)
    for i in range(1, inflight):  # (the others find the landed build at their second frame)
        step_on(i)
        step_on(i)
        jit_pending += ctxs[i].jit_wait(120000.0)
    jit_wait_ms = (time.perf_counter() - t_j) * 1e3
    # W untimed steps, continued (still untimed) until --warmup-ms of frames
    # have run: on MI355X a 1080p frame after 5 warm-up frames takes 24.6 us
    # against 22.8 us in steady state (scripts/steps_probe.sh), the clocks
    # still ramping.  Every rank runs the same count (max over ranks).
    warm_run = 0
    t_w = time.perf_counter()
    while True:
        n = max(1, args.warmup - warm_run) if warm_run < args.warmup else max(1, warm_run)
        for _ in range(n):
            step()
        warm_run += n
        torch.cuda.synchronize()
        done = warm_run >= args.warmup and (time.perf_counter() - t_w) * 1e3 >= args.warmup_ms
        if world > 1:
            flag = torch.tensor([0 if done else 1], dtype=torch.int32)
            dist.all_reduce(flag)  # gloo, host tensor: continue while any rank wants to
            done = int(flag.item()) == 0
        if done:
            break
    warm_ms_per_frame = (time.perf_counter() - t_w) * 1e3 / max(1, warm_run)

    # Device time of the K frames, from one HIP event pair on the launch
    # stream (per-launch event records cost ~6 us of GPU time per 1080p frame
    # on MI355X — they stop the next launch's waves from overlapping the
    # previous one's tail — see scripts/host_overhead.py): average = bracket / K.
    # Only a line of one frame at a time uses the bracket (its roofline launch
    # duration).  With frames in flight the bracket needs cross-stream joins at
    # both ends, which cost ~0.8 us per frame of a 20-frame region
    # (scripts/region_inflight_probe.py), and its average is a throughput, not
    # a launch's duration: the region is then the K frames and the
    # synchronize alone, and the roofline takes frame_latency_ms (below).
    # Tiled lines take their launch duration from rt_render's events.
    use_events = not tiled and inflight == 1
    bracket = timed_launches(step, streams, args.steps) if use_events else None

    def timed():
        if bracket is not None:
            return bracket()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        return None
    # The GPU should not sit idle between the warm-up and the timed region
    # (the events and the barrier above cost milliseconds): ~2 ms of untimed
    # frames keep it busy across them; the region itself is unchanged.
    burst = max(2, int(2.0 / max(warm_ms_per_frame, 1e-3)) + 1)
    for _ in range(burst):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    turn[0] = 0
    before = counters_sum()  # (a few-us copy per context: the region's rays are after - before)
    t0 = time.perf_counter()
    bracket_ms = timed()  # ends with torch.cuda.synchronize()
    # each rank's clock stops at its own synchronize; the closing barrier is
    # outside it (a gloo barrier costs ~0.1-1 ms against a 7 ms 20-frame tiled
    # region) and the max over ranks is taken below (rdist.job_totals).  In
    # tiled mode rank 0's stream holds the gather, which waits for every shard.
    elapsed = time.perf_counter() - t0
    state_after = device_state(local)
    if world > 1:
        dist.barrier()
    after = counters_sum()

    rays = after["rays"] - before["rays"]
    flops = after["algorithmic_flops"] - before["algorithmic_flops"]
    # rays per frame by kind (SURVEY.md §8d semantics; this process's GPU)
    by_kind = {k: (after[k] - before[k]) // args.steps for k in ("primary", "shadow", "reflect", "refract")}
    elapsed, total_rays = rdist.job_totals(elapsed, rays, "cpu")
    extra = {}
    if tiled:
        # per-shard render, gather + de-interleave and end-to-end device ms of
        # one frame (rt_render's events; median of 5), every rank collective
        host = np.empty((cam.height, cam.width, 3), dtype=image.cpu().numpy().dtype) if rank == 0 else None

        def lone_stats():  # one synchronous frame at a time: planned for one in flight (median of 5)
            if inflight > 1:
                ctx.set_frames_in_flight(1)
            try:
                return [ctx.render_stats(cam, args.depth, args.precision, args.out, host) for _ in range(5)]
            finally:
                if inflight > 1:
                    ctx.set_frames_in_flight(inflight)
        sts = lone_stats()
        kernel_ms = float(np.median([st["kernel_ms"] for st in sts]))
        extra = {"render_ms_per_shard": kernel_ms,
                 "gather_ms": float(np.median([st["gather_ms"] for st in sts])),
                 "frame_ms": float(np.median([st["frame_ms"] for st in sts])), "gather": args.gather}
        # both ways of assembling the frame on rank 0 (rtc.h RT_GATHER_*): the
        # line's own, then the other one over the same K steps
        variants = {args.gather: {"ms_per_step": elapsed * 1e3 / args.steps, "frame_ms": extra["frame_ms"],
                                  "gather_ms": extra["gather_ms"], "render_ms_per_shard": kernel_ms}}
        other = "peer" if args.gather == "rccl" else "rccl"
        for c in ctxs:
            c.set_gather(rtc_amd.RT_GATHER_PEER if other == "peer" else rtc_amd.RT_GATHER_RCCL)
        for _ in range(3 * inflight):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = time.perf_counter()
        timed()
        el2, _ = rdist.job_totals(time.perf_counter() - t, rays, "cpu")
        sts2 = lone_stats()
        variants[other] = {"ms_per_step": el2 * 1e3 / args.steps,
                           "frame_ms": float(np.median([st["frame_ms"] for st in sts2])),
                           "gather_ms": float(np.median([st["gather_ms"] for st in sts2])),
                           "render_ms_per_shard": float(np.median([st["kernel_ms"] for st in sts2]))}
        for c in ctxs:
            c.set_gather(rtc_amd.RT_GATHER_PEER if args.gather == "peer" else rtc_amd.RT_GATHER_RCCL)
        extra["gather_variants"] = variants
        if world > 1:
            dist.barrier()
        if rank == 0:
            # the same workload on rank 0's GPU alone (single-GPU contexts,
            # the same frames in flight)
            ones = [rtc_amd.Context(local) for _ in range(inflight)]
            try:
                for o_ in ones:
                    o_.upload(scene)
                    if inflight > 1:
                        o_.set_frames_in_flight(inflight)
                one = ones[0]
                fulls = [torch.empty((cam.height, cam.width, 3), dtype=rdtype, device="cuda") for _ in ones]
                full = fulls[0]
                turn1 = [0]

                def f1_on(i):
                    ones[i].render_device(cam, fulls[i].data_ptr(), sptrs[i], args.depth, args.precision, args.out)

                def f1n():
                    i = turn1[0]
                    turn1[0] = (i + 1) % inflight
                    f1_on(i)
                f1 = lambda: f1_on(0)  # noqa: E731
                for _ in range(max(2, args.warmup) * inflight):
                    f1n()
                torch.cuda.synchronize()
                timed1 = timed_launches(f1n, streams, args.steps)
                t1 = time.perf_counter()
                timed1()
                single_ms = (time.perf_counter() - t1) * 1e3 / args.steps
                extra["single_gpu_ms_per_step"] = single_ms
                extra["speedup_vs_1gpu"] = single_ms / (elapsed * 1e3 / args.steps)
                extra["strong_scaling_efficiency"] = extra["speedup_vs_1gpu"] / world
                # the same workload's throughput on one GPU, in the line's unit: the
                # denominator for this line's scaling (the default N=1 line is
                # configs[1], three_sphere at 1080p, a different workload)
                extra["single_gpu_value"] = total_rays / args.steps / (single_ms * 1e-3) / 1e6
                # the 8-way split on this one GPU: each shard's kernel ms (what
                # rank r renders at N = 8; warm, cost-ordered, median of 3), so
                # every line carries the slowest of 8 beside its own split
                # (each launch alone: planned for one frame in flight, as
                # frame_latency_ms is; the hint for two raises the split
                # threshold, which lengthens a lone shard: DESIGN.md §6)
                one.set_frames_in_flight(1)
                rows8 = rtc_amd.shard_rows(cam.height, 8)
                strip8 = torch.empty((rows8, cam.width, 3), dtype=rdtype, device="cuda")
                per8 = []
                for kk in range(8):
                    f8 = lambda: one.render_device(cam, strip8.data_ptr(), sptr, args.depth,  # noqa: E731
                                                   args.precision, args.out, (kk, 8))
                    for _ in range(3):
                        f8()
                    torch.cuda.synchronize()
                    per8.append(float(np.median([timed_launches(f8, stream, 1)() for _ in range(3)])))
                whole1 = float(np.median([timed_launches(f1, stream, 1)() for _ in range(3)]))
                extra["shards_of_8_on_one_gpu"] = {
                    "kernel_ms": [round(x, 4) for x in per8], "slowest_ms": max(per8),
                    "whole_frame_ms": whole1, "sum_over_whole": sum(per8) / whole1,
                    "note": "each row-block shard of the 8-way split rendered alone on rank 0's GPU (the render "
                            "time of each rank at N = 8, before the gather)"}
            finally:
                for o_ in ones:
                    o_.close()
        if world > 1:
            dist.barrier()
    elif inflight > 1:
        # The roofline's per-launch duration: the same frames one after
        # another on one stream (the K-frame bracket above overlaps frames in
        # flight, so bracket / K is the throughput, not a launch's duration;
        # rocprofv3's average duration agrees with this one).
        # (planned as a frame alone: the hint back to 1 for it, so rocprof of a
        # one-in-flight run, which the profile set is, times the same launches)
        ctx.set_frames_in_flight(1)
        lat = timed_launches(step0, [streams[0]], args.steps)
        for _ in range(burst + 8):
            step0()
        torch.cuda.synchronize()
        kernel_ms = lat() / args.steps
        ctx.set_frames_in_flight(inflight)
    else:
        kernel_ms = bracket_ms / args.steps
    line = None
    if rank == 0:
        flops_per_launch = flops / args.steps
        peak = PEAK_FP32_TFLOPS if args.precision == "f32" else PEAK_FP64_TFLOPS
        achieved = flops_per_launch / (kernel_ms * 1e-3) / 1e12
        workload = f"{args.scene}@{cam.width}x{cam.height},depth={args.depth},{args.precision}"
        if args.out == "u8":
            workload += ",u8"
        if tiled:
            # the tile split's PMC figures (scripts/shard_pmc.sh): the whole frame at
            # N = 1, one of the eight shards a rank renders at N = 8, none otherwise
            split_prof = load_profile("tile_split_pmc.json", workload + (f",shard_of_{world}" if world > 1 else ""))
            traffic = (split_prof or {}).get("traffic")
            issue = split_prof or {}
        else:
            traffic = load_profile("traffic.json", workload)
            issue = load_profile("issue.json", workload) or {}
        line = {
            "metric": "Mray/s (primary+secondary) and ms/frame at 1920x1080",
            "value": total_rays / elapsed / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_frames_run": warm_run,
            "frames_in_flight": inflight,
            # one frame's device time on its own (frames: one launch after another on
            # one stream; tiled: rank 0's render + gather + de-interleave of one frame)
            "frame_latency_ms": extra.get("frame_ms", kernel_ms) if tiled else kernel_ms,
            "rewarm_frames": burst,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if tiled else "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic: the reference's scene (scenes/%s.yaml) rendered at the configured size" % args.scene,
            "config": {"workload": workload, "scene": args.scene, "width": cam.width, "height": cam.height,
                       "max_depth": args.depth, "out": args.out,
                       "parallelism": f"{'tiles' if tiled else 'frames'}x{world}",
                       "rays_per_frame": int(total_rays // args.steps) if tiled else int(rays // args.steps),
                       "stream": args.stream,
                       "mode": "tiled" if tiled else "frames"},
            # the path is FP32-VALU bound: no MFMA, the compute roof is the vector ALU's
            "roofline": {"bound": "valu", "pipe": f"valu-{args.precision}", "achieved": achieved, "peak": peak,
                         "unit": "TFLOP/s", "frac": achieved / peak, "traffic": traffic,
                         "kernel_ms": kernel_ms, "flops_per_launch": flops_per_launch,
                         # the north star's HBM view: PMC bytes per launch over the launch time,
                         # against the ~8 TB/s memory roof (a diagnostic: the path is compute-bound)
                         "hbm_gbs": traffic / (kernel_ms * 1e-3) / 1e9 if traffic else None,
                         "hbm_frac": traffic / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS if traffic else None,
                         # the issue side (PMC, same launches): `frac` charges every ray brute force
                         # over all shapes, so culls count as achieved FLOPs; these
                         # say how busy the VALU really was and how long waves waited
                         "valu_issue_frac": issue.get("valu_issue_frac"), "wait_frac": issue.get("wait_frac")},
        }
        if tiled:
            line["roofline"]["kernel"] = "rank 0's shard launch (median of 5 instrumented frames)"
        line.update(extra)
        # clocks, power and temperature just before and just after the timed
        # region (tell a slower box from a box-sensitive build)
        line["device_state"] = {"before": state_before, "after": state_after,
                                "note": "before: ahead of the warm-up (an amdsmi query right before the "
                                        "region slows it); after: once the region's clock has stopped"}
        line["rays_by_kind"] = by_kind
        line["first_frame_ms"] = first_frame_ms
        line["first_frame_breakdown"] = phase
        try:  # per-scene build (hipRTC, or a load from RTC_JIT_CACHE) on its host thread, after the first frame
            js = ctx.jit_status()
            line["jit_build_ms"] = js["compile_ms"]
            line["jit_used"] = js["used"]
            line["jit_wait_ms"] = jit_wait_ms
            line["jit_pending"] = jit_pending
        except Exception:  # noqa: BLE001  (group contexts may not report it)
            pass
        if not tiled and world == 1:
            if ctx.scene.has_secondary() and args.depth > 0:
                # cold launch: the first frame after an upload has no recorded
                # tile costs; its tiles are handed out centre-out
                cold = []
                for _ in range(3):
                    ctx.upload(scene)
                    cold.append(timed_launches(step0, stream, 1)())
                line["cold_kernel_ms"] = float(np.median(cold))
        if not tiled and world == 1 and not args.ab:
            # a drop-in Camera::render: synchronous rt_render into host memory,
            # PCIe copy included, into a canvas kept across frames (median of
            # 10; never `value`).  A canvas allocated per call adds its first-
            # touch page faults (~0.3 ms at 1080p f32; scripts/host_frame_probe.py).
            canvas, _ = ctx.render(cam, args.depth, args.precision, args.out)
            lat = []
            for _ in range(10):
                t = time.perf_counter()
                ctx.render(cam, args.depth, args.precision, args.out, out=canvas)
                lat.append((time.perf_counter() - t) * 1e3)
            line["host_frame_ms"] = float(np.median(lat))
            # the PCIe floor of that copy: the frame's bytes at the measured
            # pinned device-to-host rate of this box's link
            pinned = torch.empty(image.shape, dtype=image.dtype, pin_memory=True)
            pinned.copy_(image, non_blocking=True)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                pinned.copy_(image, non_blocking=True)
            torch.cuda.synchronize()
            d2h_s = (time.perf_counter() - t) / 5
            line["host_frame_floor_ms"] = d2h_s * 1e3
            line["d2h_gbs"] = image.numel() * image.element_size() / d2h_s / 1e9
            # the same frame as the 8-bit canvas Canvas::to_png_file writes
            # (RT_OUT_U8: canvas.rs:117-123's quantization on the device, a
            # quarter of the bytes; INTEGRATION.md 1b'')
            if args.out != "u8":
                canvas8, _ = ctx.render(cam, args.depth, args.precision, "u8")
                lat8 = []
                for _ in range(10):
                    t = time.perf_counter()
                    ctx.render(cam, args.depth, args.precision, "u8", out=canvas8)
                    lat8.append((time.perf_counter() - t) * 1e3)
                line["host_frame_u8_ms"] = float(np.median(lat8))
                line["host_frame_u8_floor_ms"] = d2h_s * 1e3 / image.element_size()
            # rays per generation (each bounce's wavefront size):
            # one untimed diagnostic frame of the generic kernel (RT_FLAG_GENERATIONS)
            _, _, gen = ctx.render_generations(cam, args.depth, args.precision)
            light_n = len(scene.lights)
            line["rays_by_generation"] = {"traced": gen["traced"], "shaded": gen["shaded"],
                                          "shadow": [light_n * v for v in gen["shaded"]],
                                          "note": "generation g = bounce g (0 = camera rays); traced = radiance "
                                                  "rays (the wavefront), shadow = L per shaded hit"}
        if world == 1 and not tiled and not args.ab:
            line["one_shot"] = one_shot(args)
            # the same with the runtime's default copy engine (SDMA) for the frame copy
            line["one_shot_sdma_copy"] = one_shot(args, {"GPU_FORCE_BLIT_COPY_SIZE": "0"})
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene, cam, args.depth, args.cpu_seconds)
            line["cpu_baseline"]["configs0_serial"] = cpu_serial_configs0(min(3.0, args.cpu_seconds / 4))
    for c in ctxs:
        c.close()
    return line if rank == 0 else None


if __name__ == "__main__":
    main()
