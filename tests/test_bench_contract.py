"""bench.py's output contract (the driver parses this line every round).

One short run on the GPU at a small canvas: exactly one JSON line with the
metric, the whole-job value, the roofline object and the CPU baseline, and a
ray count that matches the reference's semantics for three_sphere (every
pixel hits a wall or the floor: one primary and one shadow ray per pixel).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline"}


def _run(*args, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [line for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_parses_without_a_gpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0 and "--gpus" in r.stdout and "--steps" in r.stdout


@pytest.mark.gpu
def test_bench_line_contract():
    d = _run("--steps", "20", "--warmup", "2", "--width", "320", "--height", "240", "--cpu-seconds", "0.2")
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 2 and d["higher_is_better"] is True
    assert d["unit"] == "Mray/s" and d["dtype"] == "f32" and d["scaling"] == "weak"
    assert d["config"]["rays_per_frame"] == 2 * 320 * 240
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # frames in flight (three contexts alternating) and one frame's own device time
    assert d["frames_in_flight"] == 3 and d["frame_latency_ms"] > 0
    assert d["frame_latency_ms"] == d["roofline"]["kernel_ms"]
    rl = d["roofline"]
    assert rl["unit"] == "TFLOP/s" and rl["peak"] == 157.3 and 0 < rl["frac"] < 1
    assert abs(rl["frac"] - rl["achieved"] / rl["peak"]) < 1e-12
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0
    s0 = cb["configs0_serial"]  # BASELINE configs[0]: Camera::render at 320x240, one thread
    assert s0["cores"] == 1 and s0["ms_per_frame"] > 0 and s0["rays_per_frame"] == 2 * 320 * 240
    # rays by kind and per generation
    assert d["rays_by_kind"] == {"primary": 320 * 240, "shadow": 320 * 240, "reflect": 0, "refract": 0}
    g = d["rays_by_generation"]
    assert g["traced"][0] == g["shaded"][0] == g["shadow"][0] == 320 * 240 and sum(g["traced"][1:]) == 0
    # the first frame and the one-shot (torch-free process) by phase
    fb = d["first_frame_breakdown"]
    assert {"scene_load_ms", "context_ms", "upload_ms", "first_render_ms", "d2h_ms"} <= set(fb)
    for k in ("one_shot", "one_shot_sdma_copy"):  # blit-kernel frame copy (the CLI's), runtime default (SDMA)
        os_ = d[k]
        assert os_["total_ms"] >= os_["render_ms"] > 0 and os_["context_ms"] > 0, (k, os_)
        assert os_["runs"] == 3 and len(os_["total_ms_samples"]) == 3  # median of three fresh processes
    # the strong-scaling series at every N (here N = 1): configs[3] and [4] split by the group context
    assert "NOT a scaling result" in d["scaling_note"]
    assert set(d["tile_split"]) == {"cover", "table"}
    for name, ts in d["tile_split"].items():
        assert ts["config"]["width"] == 3840 and ts["config"]["height"] == 2160 and ts["config"]["scene"] == name
        assert ts["scaling"] == "strong" and set(ts["gather_variants"]) == {"rccl", "peer"}
        for k in ("render_ms_per_shard", "single_gpu_ms_per_step", "speedup_vs_1gpu", "value"):
            assert ts[k] > 0, (name, k)


@pytest.mark.gpu
def test_bench_tiled_line_on_one_gpu():
    """--mode tiled through librtc's RCCL group with one rank (the driver's
    N > 1 default, scaled down): per-shard render, gather and end-to-end
    milliseconds and the same workload on one GPU are reported."""
    d = _run("--mode", "tiled", "--steps", "10", "--warmup", "2", "--width", "640", "--height", "360",
             "--no-cpu-baseline")
    assert KEYS <= set(d)
    assert d["scaling"] == "strong" and d["config"]["mode"] == "tiled" and d["config"]["scene"] == "cover"
    assert d["config"]["out"] == "u8" and d["config"]["parallelism"] == "tilesx1"
    for k in ("render_ms_per_shard", "gather_ms", "frame_ms", "single_gpu_ms_per_step", "speedup_vs_1gpu"):
        assert d[k] > 0, k
    assert d["roofline"]["bound"] == "valu"
    # both ways of assembling the frame on rank 0, measured over the same steps
    gv = d["gather_variants"]
    assert set(gv) == {"rccl", "peer"} and d["gather"] == "rccl"
    for v in gv.values():
        assert v["ms_per_step"] > 0 and v["frame_ms"] > 0 and v["render_ms_per_shard"] > 0


@pytest.mark.gpu
def test_bench_pool_scene_reports_cold_launch():
    d = _run("--scene", "reflect_refract", "--steps", "10", "--warmup", "2", "--width", "320", "--height", "240",
             "--no-cpu-baseline")
    assert d["cold_kernel_ms"] > 0 and d["host_frame_ms"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_frames_weak_scaling():
    """N > 1: one process per GPU (here two ranks rehearsed on the one GPU,
    BENCH_SHARE_GPU=1): each rank renders its own configs[1] frames, the line
    is the whole job's rays over the slowest rank's time, "scaling": "weak"."""
    env = dict(os.environ, BENCH_SHARE_GPU="1", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--mode", "frames", "--steps", "10", "--warmup", "2", "--width", "320",
                        "--height", "240"], capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [line for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["parallelism"] == "framesx2"
    assert d["config"]["rays_per_frame"] == 2 * 320 * 240 and "tile_split" not in d
    # the job's rays: both ranks' frames
    assert abs(d["value"] * d["ms_per_step"] * 1e-3 - 2 * 2 * 320 * 240 / 1e6) < 1e-6 * d["value"]
