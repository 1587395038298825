"""Per-scene kernels (csrc/rtc_jit.cpp) against the generic kernels.

For f32 frames the library compiles the tracer source once per uploaded
world with the shape table as compile-time constants (hipRTC).  Same source,
same operations, same values: every frame must equal the generic kernel's
bit for bit, counters included, for every reference scene and for a world
with every shape and pattern kind.  (Parity with the oracle then carries
over from tests/test_gpu_parity.py, which runs the generic kernels; at the
bench's own sizes tests/test_gpu_fullsize.py builds the per-scene kernels
in line (RT_JIT_SYNC), asserts they ran, and checks their frames against
both the generic kernel and the oracle.)
"""
import numpy as np
import pytest

from conftest import scene_fixture

pytestmark = pytest.mark.gpu

# the BASELINE configs' scenes (bench.py lines)
BENCH_SCENES = ("three_sphere_scene", "reflect_refract", "cover", "table")
SCENES = ["three_sphere_scene", "reflect_refract", "cover", "table", "cylinders", "metal", "refraction",
          "shadow_puppets"]


def _counts(st):
    return {k: st[k] for k in ("primary", "shadow", "reflect", "refract", "shaded", "lit_patterned",
                               "refract_evals", "schlick_evals")}


def _both(gpu_ctx, tables, cam, depth=6):
    """(generic frame, stats, per-scene frame, stats, repeat) — the per-scene
    frame is None when the library declined to use its build (pool-kernel
    worlds, or a build that spills; jit_status() says why)."""
    gpu_ctx.upload(tables)
    gpu_ctx.set_jit(0)
    a, sa = gpu_ctx.render(cam, depth, precision="f32")
    assert not gpu_ctx.jit_status()["used"]
    gpu_ctx.set_jit(1)
    try:
        b, sb = gpu_ctx.render(cam, depth, precision="f32")
        st = gpu_ctx.jit_status()
        if not st["used"]:
            assert depth > 0 and tables.has_secondary() or "not used" in st["log"], st["log"][:2000]
            return a, sa, None, None, None
        b2, _ = gpu_ctx.render(cam, depth, precision="f32")
    finally:
        gpu_ctx.set_jit(2)
    return a, sa, b, sb, b2





@pytest.mark.parametrize("name", SCENES)
@pytest.mark.parametrize("depth", [0, 6])
def test_per_scene_kernel_is_bit_identical(gpu_ctx, rtc, name, depth):
    """Depth 0 runs the direct kernel on every scene (no child rays)."""
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 320, 200)
    a, sa, b, sb, b2 = _both(gpu_ctx, scene, cam, depth)
    if name in BENCH_SCENES:
        # the bench workloads must keep their per-scene kernels: a change that
        # makes a build spill (refused, generic kernel) would otherwise only
        # show up as a slower bench
        assert b is not None, f"{name} fell back to the generic kernel: {gpu_ctx.jit_status()['log'][:400]}"
    if b is None:
        return
    assert np.array_equal(a, b) and np.array_equal(a, b2), f"{name}: {int((a != b).any(axis=2).sum())} px differ"
    assert _counts(sa) == _counts(sb)


@pytest.mark.parametrize("depth", [0, 6])
def test_per_scene_kernel_all_kinds(gpu_ctx, depth):
    """Every shape and pattern kind (a complex pattern's sub-patterns
    included: the per-scene build compiles only the kinds its world holds),
    glass, two lights: the per-scene frame equals the generic one."""
    from test_gpu_parity import _all_shapes_world
    from rtc_amd import world as W
    cam = W.camera(160, 120, 1.0, (0, 3, -8), (0, 0.8, 0), (0, 1, 0))
    a, sa, b, sb, _ = _both(gpu_ctx, _all_shapes_world(), cam, depth)
    if b is not None:
        assert np.array_equal(a, b) and _counts(sa) == _counts(sb)


def test_per_scene_kernel_complex_pattern_only(gpu_ctx):
    """A world whose only material pattern is a complex one: its stripe and
    checker sub-patterns must be compiled into the per-scene build."""
    from rtc_amd import world as W
    pat = W.complex_pattern(W.stripe_pattern((1, 1, 1), (0, 0, 0)), W.checker_pattern((1, 0, 0), (0, 1, 0)))
    shapes = [W.plane(W.Material(reflectiveness=0.4)),
              W.sphere(W.Material(pattern=pat), W.mat_mul(W.translation(0, 1, 0), W.scaling(1.5, 1.5, 1.5)))]
    tables = W.World([W.Light((-10, 10, -10))], shapes).tables()
    cam = W.camera(160, 120, 1.0, (0, 2, -6), (0, 1, 0), (0, 1, 0))
    for depth in (0, 6):
        a, sa, b, sb, _ = _both(gpu_ctx, tables, cam, depth)
        if b is not None:
            assert np.array_equal(a, b) and _counts(sa) == _counts(sb)


def _fresh_world(rtc, name, salt):
    """A scene whose shape table no earlier test uploaded (the per-process
    build cache would otherwise hand over a finished build at once): the
    reference scene plus one tiny sphere far behind the camera."""
    import ctypes as C
    scene = scene_fixture(name)
    n = len(scene.shapes)
    shapes = (rtc.ShapeDesc * (n + 1))()
    C.memmove(shapes, scene.shapes, n * C.sizeof(rtc.ShapeDesc))
    extra = shapes[n]
    C.pointer(extra)[0] = scene.shapes[0]
    extra.kind = rtc.SHAPE_KINDS["sphere"]
    # inverse of translation(0, 1000 + salt, -1e4) * scaling(0.01, 0.01, 0.01)
    inv = [100.0, 0, 0, 0, 0, 100.0, 0, -100.0 * (1000.0 + salt), 0, 0, 100.0, 1e6, 0, 0, 0, 1.0]
    for i, v in enumerate(inv):
        extra.inverse[i] = v
    scene.shapes = shapes
    return scene


def test_auto_mode_builds_off_the_frame_path(rtc):
    """RT_JIT_AUTO (the default): the first large frame of an upload renders
    with the generic kernel and starts nothing (a one-shot render never
    compiles); the second starts the build on a host thread and still renders
    generic; once the build lands the next frame switches.  Every frame,
    before and after the switch, is the same bit for bit."""
    import time
    scene = _fresh_world(rtc, "three_sphere_scene", 1.0)
    cam = rtc.camera_resize(scene.camera, 640, 480)
    with rtc.Context(0) as ctx:
        ctx.upload(scene)
        ctx.render(rtc.camera_resize(scene.camera, 64, 64), 6, precision="f32")  # small: never built
        t = time.perf_counter()
        a, sa = ctx.render(cam, 6, precision="f32")
        first_ms = (time.perf_counter() - t) * 1e3
        assert not ctx.jit_status()["used"] and ctx.jit_status()["compile_ms"] == 0
        assert ctx.jit_wait(0) == 0  # the first large frame started no build
        t = time.perf_counter()
        b, sb = ctx.render(cam, 6, precision="f32")  # starts the build, renders generic
        second_ms = (time.perf_counter() - t) * 1e3
        assert not ctx.jit_status()["used"]
        assert ctx.jit_wait(60000) == 0
        c, sc = ctx.render(cam, 6, precision="f32")
        st = ctx.jit_status()
        assert st["used"], st["log"][:2000]
        assert st["compile_ms"] > 0
        assert np.array_equal(a, b) and np.array_equal(a, c)
        assert _counts(sa) == _counts(sb) == _counts(sc)
        # neither generic frame waited for hipRTC (a build takes 300-1300 ms)
        assert first_ms < 250 and second_ms < 250, (first_ms, second_ms)
        ctx.render(cam, 6, precision="f64")
        assert not ctx.jit_status()["used"]  # the f64 parity path is never rebuilt


def test_eager_mode_and_reupload_reuse(rtc):
    """RT_JIT_EAGER starts the build at the first large frame; a re-upload of
    the same world (another context too) picks the finished build up at once."""
    scene = _fresh_world(rtc, "shadow_puppets", 2.0)
    cam = rtc.camera_resize(scene.camera, 640, 480)
    with rtc.Context(0) as ctx:
        ctx.set_jit(rtc.RT_JIT_EAGER)
        ctx.upload(scene)
        a, _ = ctx.render(cam, 6, precision="f32")
        assert ctx.jit_wait(60000) == 0
        b, _ = ctx.render(cam, 6, precision="f32")
        assert ctx.jit_status()["used"] and np.array_equal(a, b)
    with rtc.Context(0) as ctx:  # default mode, a new context: the process already holds the build
        ctx.upload(scene)
        c, _ = ctx.render(cam, 6, precision="f32")
        assert ctx.jit_status()["used"] and np.array_equal(a, c)
        assert ctx.jit_status()["compile_ms"] == 0  # built by the other context


def test_destroy_with_a_build_in_flight(rtc):
    """A context destroyed while its build compiles does not wait for it and
    leaves nothing broken: the build lands for the next context of the world."""
    scene = _fresh_world(rtc, "three_sphere_scene", 3.0)
    cam = rtc.camera_resize(scene.camera, 640, 480)
    ctx = rtc.Context(0)
    ctx.set_jit(rtc.RT_JIT_EAGER)
    ctx.upload(scene)
    a, _ = ctx.render(cam, 6, precision="f32")
    ctx.close()
    with rtc.Context(0) as c2:
        c2.set_jit(rtc.RT_JIT_SYNC)  # waits for the build in flight instead of starting another
        c2.upload(scene)
        b, _ = c2.render(cam, 6, precision="f32")
        assert c2.jit_status()["used"] and np.array_equal(a, b)


_EXIT_PROBE = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ray-tracer-challenge-rs_amd"))
import rtc_amd
from rtc_amd import scene_io
scene = scene_io.load(os.path.join(sys.argv[1], "tests", "golden", "scenes", "cover.json"))
cam = rtc_amd.camera_resize(scene.camera, 640, 360)
ctx = rtc_amd.Context(0)
ctx.set_jit(int(sys.argv[2]))
ctx.upload(scene)
img, st = ctx.render(cam, 6, precision="f32")
js = ctx.jit_status()
print(json.dumps({"used": js["used"], "ms": js["compile_ms"], "rays": st["rays"]}), flush=True)
"""  # exits with the per-scene build (when started) still compiling


def test_exit_with_a_build_in_flight(tmp_path):
    """A host that exits while its per-scene build compiles exits cleanly (the
    compile runs in a child process, csrc/rtc_jitc.cpp; on a thread it had
    corrupted the heap at exit), and the build still lands in the disk cache
    for the next process."""
    import json
    import os
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cache = tmp_path / "cache"
    env = dict(os.environ, RTC_JIT_CACHE=str(cache))

    def run(mode):
        out = subprocess.run([sys.executable, "-c", _EXIT_PROBE, root, str(mode)], env=env, capture_output=True,
                             text=True, timeout=100)
        assert out.returncode == 0, out.stderr[-2000:]
        return json.loads(out.stdout.strip().splitlines()[-1])

    first = run(3)  # RT_JIT_EAGER: the build starts at this frame, the process exits at once
    assert not first["used"]
    # (a pool world compiles two builds, at 7 waves/SIMD and at the static
    # occupancy: rtc_jit.cpp jit_function; both must land)
    deadline = time.time() + 90
    def landed():
        return sum(p.suffix == ".co" for p in cache.iterdir()) if cache.exists() else 0
    while time.time() < deadline and landed() < 2:
        time.sleep(0.2)
    assert landed() >= 2, "the orphaned compiles did not land in the cache"
    second = run(3)  # the build comes from the disk cache at the first frame
    assert second["used"] and second["rays"] == first["rays"]
    assert second["ms"] < 100, second


def test_failed_launch_keeps_the_queue_heads(gpu_ctx, rtc):
    """A pool launch that fails after planning (RT_FLAG_FAIL_LAUNCH) must not
    consume a set of queue heads: the next frame is complete and equal."""
    scene = scene_fixture("reflect_refract")
    cam = rtc.camera_resize(scene.camera, 320, 200)
    gpu_ctx.upload(scene)
    a, sa = gpu_ctx.render(cam, 6, precision="f32")
    import torch
    img = torch.zeros((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        with pytest.raises(rtc.RenderError):
            gpu_ctx.render_device(cam, img.data_ptr(), s, 6, "f32", "real", (0, 1), rtc.RT_FLAG_FAIL_LAUNCH)
        b, sb = gpu_ctx.render(cam, 6, precision="f32")
        assert np.array_equal(a, b) and _counts(sa) == _counts(sb)


_CACHE_PROBE = r"""
import hashlib, json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ray-tracer-challenge-rs_amd"))
import rtc_amd
from rtc_amd import scene_io
scene = scene_io.load(os.path.join(sys.argv[1], "tests", "golden", "scenes", "three_sphere_scene.json"))
cam = rtc_amd.camera_resize(scene.camera, 320, 200)
with rtc_amd.Context(0) as ctx:
    ctx.upload(scene)
    ctx.set_jit(1)
    img, st = ctx.render(cam, 5, precision="f32")
    js = ctx.jit_status()
print(json.dumps({"used": js["used"], "ms": js["compile_ms"], "rays": st["rays"],
                  "sha": hashlib.sha256(img.tobytes()).hexdigest()}))
"""


def test_per_scene_build_disk_cache(tmp_path):
    """A second process loads the first one's per-scene build from the
    RTC_JIT_CACHE directory instead of compiling it: same frame, bit for bit,
    and no compile time."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # comgr keeps a compile cache of its own (on by default): a fresh one, so
    # the first process really compiles
    env = dict(os.environ, RTC_JIT_CACHE=str(tmp_path / "cache"), AMD_COMGR_CACHE_DIR=str(tmp_path / "comgr"))

    def run():
        out = subprocess.run([sys.executable, "-c", _CACHE_PROBE, root], env=env, capture_output=True, text=True,
                             timeout=100)
        assert out.returncode == 0, out.stderr[-2000:]
        return json.loads(out.stdout.strip().splitlines()[-1])

    first = run()
    files = sorted(p.name for p in (tmp_path / "cache").iterdir())
    second = run()
    assert first["used"] and second["used"]
    assert len(files) == 1 and files[0].endswith(".co"), files
    assert first["sha"] == second["sha"] and first["rays"] == second["rays"]
    # a hipRTC build of the direct kernel takes ~300 ms; a cache load a few ms
    assert first["ms"] > 50 and second["ms"] < 0.25 * first["ms"], (first["ms"], second["ms"])
    # a damaged file (truncated code object) is rebuilt and rewritten, not trusted
    f = tmp_path / "cache" / files[0]
    size = f.stat().st_size
    with open(f, "r+b") as fh:
        fh.truncate(size // 2)
    third = run()
    assert third["used"] and third["sha"] == first["sha"], third
    assert f.stat().st_size == size
