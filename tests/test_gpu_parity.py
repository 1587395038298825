"""GPU parity: the HIP render path (through the C-ABI) against the f64 oracle.

Tolerances (the f64 -> f32 statement of DESIGN.md §Parity):
  * precision f64 — the reference's operation order, FMA sites and
    EPSILON = 8e-8: every pixel within ABS64 = 1e-9 of the oracle, ray counters
    identical.  (The only differences are the GPU libm pow and the order in
    which the tree's weighted contributions are summed.)
  * precision f32 — per scene, the observed agreement with the oracle plus a
    stated margin (tests/f32_tolerance.py: pixels within 2/255 after 8-bit
    quantization, canvas.rs:117-123, mean |err|, each ray kind and the total).
"""
import math

import numpy as np
import pytest

import f32_tolerance
from conftest import scene_fixture

pytestmark = pytest.mark.gpu

ABS64 = 1e-9
F32_PIX_FRAC = 0.99   # worlds other than the reference scenes (KAT and all-kinds worlds)
SQ2 = math.sqrt(2.0)

SCENES = ["three_sphere_scene", "reflect_refract", "cover", "table", "cylinders", "metal", "refraction",
          "shadow_puppets"]


def _pix_agree(a, b, oracle, lsb=2):
    d = np.abs(oracle.quantize(a).astype(int) - oracle.quantize(b).astype(int)).max(axis=2)
    return float((d <= lsb).mean())


def _counts(st):
    return {k: st[k] for k in ("primary", "shadow", "reflect", "refract", "shaded", "lit_patterned",
                               "refract_evals", "schlick_evals")}


# ------------------------------------------------- reference KAT worlds
def _kat_world(name):
    from rtc_amd import world as W
    w = W.World.default()
    if name == "behind_ray":  # world.rs:315-334
        w.shapes[0].material.ambient = 1.0
        w.shapes[1].material.ambient = 1.0
    elif name in ("transparent", "reflective_transparent"):  # world.rs:573-629
        fm = W.Material(transparency=0.5, refractive_index=1.5)
        if name == "reflective_transparent":
            fm.reflectiveness = 0.5
        w.shapes.append(W.plane(fm, W.translation(0, -1, 0)))
        w.shapes.append(W.sphere(W.Material(color=(1, 0, 0), ambient=0.5), W.translation(0, -3.5, -0.5)))
    elif name == "reflective_plane":  # world.rs:427-447
        w.shapes.append(W.plane(W.Material(reflectiveness=0.5), W.translation(0, -1, 0)))
    elif name == "mirrors":  # world.rs:449-466
        w = W.World([W.Light((0, 0, 0))], [W.plane(W.Material(reflectiveness=1.0), W.translation(0, -1, 0)),
                                            W.plane(W.Material(reflectiveness=1.0), W.translation(0, 1, 0))])
    return w.tables()


KAT_RAYS = [
    # (world, ray, depth, expected, src)
    ("default", (0, 0, -5, 0, 0, 1), 6, (0.38066119308103435, 0.47582649135129296, 0.28549589481077575),
     "world.rs:302-313"),
    ("default", (0, 0, -5, 0, 1, 0), 6, (0.0, 0.0, 0.0), "world.rs:294-300"),
    ("behind_ray", (0, 0, 0.75, 0, 0, -1), 6, (1.0, 1.0, 1.0), "world.rs:315-334"),
    ("transparent", (0, 0, -3, 0, -SQ2 / 2, SQ2 / 2), 5,
     (0.9364253889815014, 0.6864253889815014, 0.6864253889815014), "world.rs:573-599"),
    ("reflective_transparent", (0, 0, -3, 0, -SQ2 / 2, SQ2 / 2), 5,
     (0.9339151412754023, 0.696434227200244, 0.692430691912747), "world.rs:601-629"),
    ("reflective_plane", (0, 0, -3, 0, -SQ2 / 2, SQ2 / 2), 1,
     (0.8767560027604027, 0.9243386562051279, 0.8291733493156773), "world.rs:427-447"),
]


@pytest.mark.parametrize("precision,tol", [("f64", 1e-9), ("f32", 2e-4)])
@pytest.mark.parametrize("case", range(len(KAT_RAYS)))
def test_reference_known_answers_through_color_at(gpu_ctx, oracle, case, precision, tol):
    wname, ray, depth, expected, src = KAT_RAYS[case]
    tables = _kat_world(wname)
    gpu_ctx.upload(tables)
    got, st = gpu_ctx.color_at([ray], depth=depth, precision=precision)
    orc, ost = oracle.color_at(tables, [ray], depth=depth)
    # the reference asserts these with coarse_eq (|err| < EPSILON = 8e-8)
    assert np.allclose(orc[0], expected, atol=8e-8, rtol=0), f"oracle vs reference ({src})"
    assert np.abs(got[0] - np.array(expected)).max() < max(tol, 8e-8), f"{precision} {got[0]} vs {expected} ({src})"
    assert np.abs(got[0] - orc[0]).max() < tol, f"{precision} {got[0]} vs oracle {orc[0]} ({src})"
    if precision == "f64":
        assert _counts(st) == _counts(ost)


def test_mirrors_terminate(gpu_ctx, oracle):
    """world.rs:449-466: two parallel mirrors; the depth bound ends the recursion."""
    tables = _kat_world("mirrors")
    gpu_ctx.upload(tables)
    got, st = gpu_ctx.color_at([(0, 0, 0, 0, 1, 0)], depth=6, precision="f64")
    orc, ost = oracle.color_at(tables, [(0, 0, 0, 0, 1, 0)], depth=6)
    assert np.abs(got - orc).max() < ABS64
    assert st["reflect"] == 6 and _counts(st) == _counts(ost)


def test_color_at_random_rays_default_world(gpu_ctx, oracle):
    from rtc_amd import world as W
    tables = W.World.default().tables()
    rng = np.random.default_rng(1234)
    o = rng.uniform(-3, 3, size=(4096, 3))
    d = rng.normal(size=(4096, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], axis=1)
    gpu_ctx.upload(tables)
    got, st = gpu_ctx.color_at(rays, precision="f64")
    orc, ost = oracle.color_at(tables, rays)
    assert np.abs(got - orc).max() < ABS64
    assert _counts(st) == _counts(ost)


# ------------------------------------------------------- reference scenes
@pytest.mark.parametrize("name", SCENES)
def test_scene_parity_f64(gpu_ctx, oracle, rtc, name):
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 96, 64)
    gpu_ctx.upload(scene)
    img, st = gpu_ctx.render(cam, 6, precision="f64")
    ref, rst = oracle.render(scene, cam, 6, threads=8)
    err = np.abs(img - ref)
    assert err.max() < ABS64, f"{name}: max |err| {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
    assert _counts(st) == _counts(rst)


@pytest.mark.parametrize("name", SCENES)
def test_scene_parity_f32(gpu_ctx, oracle, rtc, name):
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 160, 120)
    gpu_ctx.upload(scene)
    img, st = gpu_ctx.render(cam, 6, precision="f32")
    ref, rst = oracle.render(scene, cam, 6, threads=8)
    agree = _pix_agree(img, ref, oracle)
    mean = float(np.abs(img.astype(np.float64) - ref).mean())
    f32_tolerance.check(name, agree, mean, st, rst, cam.width * cam.height)


def test_headline_config_full_size(gpu_ctx, oracle, rtc):
    """BASELINE configs[1]: three_sphere_scene at 1920x1080, every pixel hits
    a wall or the floor, so rays/frame = primary + shadow = 2*W*H exactly."""
    scene = scene_fixture("three_sphere_scene")
    cam = rtc.camera_resize(scene.camera, 1920, 1080)
    gpu_ctx.upload(scene)
    img, st = gpu_ctx.render(cam, 6, precision="f32")
    assert st["primary"] == 1920 * 1080 and st["shadow"] == 1920 * 1080 and st["reflect"] == 0
    img2, _ = gpu_ctx.render(cam, 6, precision="f32")
    assert np.array_equal(img, img2), "render is not deterministic"
    ref, _ = oracle.render(scene, cam, 6, threads=16)
    assert _pix_agree(img, ref, oracle) >= 0.999


@pytest.mark.parametrize("name", ["reflect_refract", "table"])
def test_pool_determinism_and_u8(gpu_ctx, rtc, oracle, name):
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 200, 150)
    gpu_ctx.upload(scene)
    a, sa = gpu_ctx.render(cam, 6, precision="f32")
    b, sb = gpu_ctx.render(cam, 6, precision="f32")
    assert np.array_equal(a, b) and _counts(sa) == _counts(sb)
    q, _ = gpu_ctx.render(cam, 6, precision="f32", out_format="u8")
    assert np.array_equal(q, oracle.quantize(a.astype(np.float64)))


def _render_with_env(rtc, monkeypatch, env, scene, cam, precision):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with rtc.Context(0) as c:
        c.upload(scene)
        return c.render(cam, 6, precision=precision)


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("name", ["three_sphere_scene", "shadow_puppets", "cover", "table", "cylinders", "metal"])
def test_cull_is_exact(gpu_ctx, rtc, monkeypatch, name, precision):
    """The wave cull is acceleration only: the frame with the cull off
    (RTC_DEBUG=cull=0: every shape uploaded as unbounded) equals the default frame
    bit for bit, counters included."""
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 320, 200)
    gpu_ctx.upload(scene)
    a, sa = gpu_ctx.render(cam, 6, precision=precision)
    b, sb = _render_with_env(rtc, monkeypatch, {"RTC_DEBUG": "cull=0"}, scene, cam, precision)
    assert np.array_equal(a, b), f"{name} {precision}: the cull changed {int((a != b).any(axis=2).sum())} px"
    assert _counts(sa) == _counts(sb)


@pytest.mark.parametrize("name", ["reflect_refract", "refraction"])
def test_kind_variant_is_exact(gpu_ctx, rtc, monkeypatch, name):
    """Worlds of spheres and planes run the pool kernel built with only those
    kinds' loops (rtc_kernels_sp.o): the same frame, bit for bit, as the
    all-kinds kernel (RTC_DEBUG=kind_variants=0), counters included."""
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 256, 160)
    gpu_ctx.upload(scene)
    a, sa = gpu_ctx.render(cam, 6, precision="f32")
    b, sb = _render_with_env(rtc, monkeypatch, {"RTC_DEBUG": "kind_variants=0"}, scene, cam, "f32")
    assert np.array_equal(a, b) and _counts(sa) == _counts(sb)


@pytest.mark.parametrize("name", ["reflect_refract", "cover"])
def test_cost_ordered_schedule_is_exact(gpu_ctx, rtc, monkeypatch, name):
    """Repeated launches of one frame run heaviest-tile-first from the last
    launch's per-tile costs (order_tiles): scheduling only — every ordered
    render equals the raster-ordered render of a context with RTC_DEBUG=tile_order=0."""
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 256, 160)
    gpu_ctx.upload(scene)
    first, s1 = gpu_ctx.render(cam, 6, precision="f32")  # raster order, records costs
    for _ in range(2):                                   # cost-ordered
        img, st = gpu_ctx.render(cam, 6, precision="f32")
        assert np.array_equal(img, first) and _counts(st) == _counts(s1)
    raster, s0 = _render_with_env(rtc, monkeypatch, {"RTC_DEBUG": "tile_order=0"}, scene, cam, "f32")
    assert np.array_equal(raster, first) and _counts(s0) == _counts(s1)


@pytest.mark.parametrize("shard", [(0, 1), (1, 4)])
@pytest.mark.parametrize("name", ["reflect_refract", "cover"])
def test_split_tiles_are_exact(rtc, monkeypatch, name, shard):
    """Heavy tiles handed out in 2, 4, 8 or 16 parts (order_tiles; split tiny
    splits nearly every tile 4 (split_max=3: 8, 4: 16) ways, at 1 every tile above the mean load),
    then the frozen order reused (launches 4 and 5): every render equals the
    raster-ordered one bit for bit, counters included.  The first launch runs
    the centre-out cold order, later ones the costliest items at raised wave
    priority."""
    scene = scene_fixture(name)
    cam = rtc.camera_resize(scene.camera, 256, 160)
    rows = rtc.shard_rows(cam.height, shard[1])
    raster, s0 = _render_with_env(rtc, monkeypatch, {"RTC_DEBUG": "tile_order=0"}, scene, cam, "f32")
    raster = raster[:rows] if shard[1] == 1 else None
    for split, most in (("0.0001", "2"), ("1", "2"), ("0.0001", "3"), ("0.0001", "4"), ("1", "4")):
        # up to 4, 8 (half-wave seeds) or 16 parts (wave-row seeds)
        monkeypatch.setenv("RTC_DEBUG", f"tile_order=1,split={split},split_max={most}")
        with rtc.Context(0) as c:
            c.upload(scene)
            first, s1 = c.render(cam, 6, precision="f32", shard=shard)
            if raster is not None:
                assert np.array_equal(first, raster) and _counts(s1) == _counts(s0)
            for _ in range(4):
                img, st = c.render(cam, 6, precision="f32", shard=shard)
                assert np.array_equal(img, first) and _counts(st) == _counts(s1)


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_cull_is_exact_for_grazing_rays(gpu_ctx, rtc, monkeypatch, precision):
    """Rays aimed within 1e-6 of sphere and cube silhouettes (rt_color_at
    culls every bounded shape): identical with and without the cull."""
    from rtc_amd import world as W
    w = W.World([W.Light((-10, 10, -10))],
                [W.sphere(W.Material(color=(1, 0.2, 0.2)), W.mat_mul(W.translation(0.3, 0.1, 0), W.scaling(0.7, 1.3, 0.9))),
                 W.cube(W.Material(color=(0.2, 1, 0.2)), W.translation(2.5, 0, 0.5))])
    tables = w.tables()
    rng = np.random.default_rng(7)
    n = 8192
    o = rng.uniform(-6, 6, size=(n, 3))
    o[:, 2] = -8
    # targets on (or 1e-6 off) the unit sphere / cube surface in object space
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    u *= 1.0 + rng.choice([-1e-6, 0.0, 1e-6], size=(n, 1))
    sph = np.array([0.3, 0.1, 0]) + u * np.array([0.7, 1.3, 0.9])
    cub = np.array([2.5, 0, 0.5]) + np.clip(u * 1.8, -1 - 1e-6, 1 + 1e-6)
    tgt = np.where(rng.random((n, 1)) < 0.5, sph, cub)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], axis=1)
    gpu_ctx.upload(tables)
    a, sa = gpu_ctx.color_at(rays, precision=precision)
    monkeypatch.setenv("RTC_DEBUG", "cull=0")
    with rtc.Context(0) as c:
        c.upload(tables)
        b, sb = c.color_at(rays, precision=precision)
    assert np.array_equal(a, b) and _counts(sa) == _counts(sb)


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_shards_reassemble_to_the_full_frame(gpu_ctx, rtc, shards):
    import torch
    scene = scene_fixture("cover")
    cam = rtc.camera_resize(scene.camera, 200, 136)  # 136 = 8.5 tile rows: ragged last tile row
    gpu_ctx.upload(scene)
    full, st_full = gpu_ctx.render(cam, 6, precision="f32")
    rows = rtc.shard_rows(cam.height, shards)
    strips = [gpu_ctx.render(cam, 6, precision="f32", shard=(s, shards))[0] for s in range(shards)]
    for s in strips:
        assert s.shape == (rows, cam.width, 3)
    gathered = torch.from_numpy(np.concatenate(strips, axis=0)).cuda()
    image = torch.zeros((cam.height, cam.width, 3), dtype=torch.float32, device="cuda")
    gpu_ctx.assemble_shards(gathered.data_ptr(), cam.width, cam.height, shards, 12, image.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(image.cpu().numpy(), full)


@pytest.mark.parametrize("w,h", [(1, 1), (17, 5), (33, 31)])
def test_ragged_canvas_sizes(gpu_ctx, oracle, rtc, w, h):
    scene = scene_fixture("reflect_refract")
    cam = rtc.camera_resize(scene.camera, w, h)
    gpu_ctx.upload(scene)
    img, st = gpu_ctx.render(cam, 6, precision="f64")
    ref, rst = oracle.render(scene, cam, 6)
    assert img.shape == (h, w, 3) and np.abs(img - ref).max() < ABS64
    assert _counts(st) == _counts(rst)


@pytest.mark.parametrize("depth", [0, 1, 2, 5])
def test_depth_cutoffs(gpu_ctx, oracle, rtc, depth):
    scene = scene_fixture("reflect_refract")
    cam = rtc.camera_resize(scene.camera, 48, 32)
    gpu_ctx.upload(scene)
    img, st = gpu_ctx.render(cam, depth, precision="f64")
    ref, rst = oracle.render(scene, cam, depth)
    assert np.abs(img - ref).max() < ABS64
    assert _counts(st) == _counts(rst)


def test_empty_world_and_no_lights(gpu_ctx, oracle, rtc):
    from rtc_amd import world as W
    cam = W.camera(32, 16, math.pi / 2, (0, 0, -5), (0, 0, 0), (0, 1, 0))
    empty = W.World([W.Light((-10, 10, -10))], []).tables()
    gpu_ctx.upload(empty)
    img, st = gpu_ctx.render(cam, 6, precision="f32")
    assert not img.any() and st["shaded"] == 0
    dark = W.World([], W.World.default().shapes).tables()
    gpu_ctx.upload(dark)
    img, st = gpu_ctx.render(cam, 6, precision="f64")
    ref, _ = oracle.render(dark, cam, 6)
    assert np.abs(img - ref).max() < ABS64 and st["shadow"] == 0


def _all_shapes_world():
    """Every shape kind (cylinder/cone/triangle are in no config scene) plus
    every pattern kind, reflective and transparent materials."""
    from rtc_amd import world as W
    checker = W.checker_pattern((0.2, 0.2, 0.2), (0.9, 0.9, 0.9)).set_transformation(W.scaling(0.5, 0.5, 0.5))
    shapes = [
        W.plane(W.Material(pattern=checker, reflectiveness=0.3)),
        W.sphere(W.Material.glass(), W.translation(-1.5, 1, 0)),
        W.cube(W.Material(color=(0.8, 0.3, 0.3), pattern=W.stripe_pattern((1, 0, 0), (0, 0, 1))),
               W.mat_mul(W.translation(1.5, 0.5, 1), W.scaling(0.5, 0.5, 0.5))),
        W.cylinder(0, 1.5, True, W.Material(color=(0.2, 0.8, 0.2), reflectiveness=0.5),
                   W.mat_mul(W.translation(0, 0, 2.5), W.scaling(0.6, 1, 0.6))),
        W.cylinder(0, 0.5, False, W.Material(pattern=W.ring_pattern((1, 1, 0), (0, 1, 1))),
                   W.translation(2.5, 0, -1)),
        W.cone(-1, 0, True, W.Material(pattern=W.gradient_pattern((1, 0, 1), (0, 1, 0)), transparency=0.6,
                                       refractive_index=1.3), W.mat_mul(W.translation(-2.5, 1, 2), W.scaling(0.7, 1, 0.7))),
        W.triangle((-1, 0.2, -1), (1, 0.2, -1.5), (0, 2, -1.2), W.Material(color=(0.9, 0.9, 0.2), reflectiveness=0.2)),
        W.sphere(W.Material(pattern=W.complex_pattern(W.stripe_pattern((1, 1, 1), (0, 0, 0)),
                                                      W.checker_pattern((1, 0, 0), (0, 1, 0)))),
                 W.mat_mul(W.translation(0.5, 0.4, -2.5), W.scaling(0.4, 0.4, 0.4))),
    ]
    lights = [W.Light((-10, 10, -10)), W.Light((5, 8, -6), (0.3, 0.3, 0.4))]
    return W.World(lights, shapes).tables()


def test_all_shape_and_pattern_kinds(gpu_ctx, oracle):
    from rtc_amd import world as W
    tables = _all_shapes_world()
    cam = W.camera(120, 90, 1.0, (0, 3, -8), (0, 0.8, 0), (0, 1, 0))
    gpu_ctx.upload(tables)
    img, st = gpu_ctx.render(cam, 6, precision="f64")
    ref, rst = oracle.render(tables, cam, 6, threads=8)
    assert np.abs(img - ref).max() < ABS64
    assert _counts(st) == _counts(rst)
    img32, _ = gpu_ctx.render(cam, 6, precision="f32")
    assert _pix_agree(img32, ref, oracle) >= F32_PIX_FRAC


def test_consecutive_launches_keep_queue_epochs(gpu_ctx, rtc):
    """Tile queues are cumulative device counters shared by every launch of a
    context; alternating canvas sizes, kernels and precisions must reproduce
    the same frames and counters exactly."""
    scene = scene_fixture("reflect_refract")
    gpu_ctx.upload(scene)
    # 1920x1080 has more tiles than resident workgroups (the direct kernel's
    # static stride runs several rounds, the pool kernel's queues hand out
    # tiles by atomics); the small canvases fit in one round
    cams = [rtc.camera_resize(scene.camera, w, h)
            for (w, h) in ((37, 29), (1920, 1080), (200, 100), (16, 16), (1000, 700), (1, 7))]
    first = {}
    for rnd in range(3):
        for i, cam in enumerate(cams):
            for depth in (0, 6):  # depth 0 runs the direct kernel, 6 the pool kernel
                for prec in ("f32", "f64"):
                    img, st = gpu_ctx.render(cam, depth, precision=prec)
                    key = (i, depth, prec)
                    if rnd == 0:
                        first[key] = (img, _counts(st))
                    else:
                        assert np.array_equal(img, first[key][0]) and _counts(st) == first[key][1], key
                    assert st["primary"] == cam.width * cam.height


@pytest.mark.parametrize("name", ["reflect_refract", "cover"])
def test_moved_camera_reuses_order_exactly(gpu_ctx, rtc, monkeypatch, name):
    """A moved camera starts from the previous camera's tile order (plan_tile_order):
    scheduling only — every frame along the path equals its raster-ordered render."""
    scene = scene_fixture(name)
    base = rtc.camera_resize(scene.camera, 256, 160)
    view = np.linalg.inv(np.array(list(base.inverse)).reshape(4, 4))
    cams = []
    for k in range(3):
        shift = np.eye(4)
        shift[0, 3] = 0.05 * k
        cams.append(rtc.camera_set_transform(base, shift @ view))
    gpu_ctx.upload(scene)
    ordered = []
    for c in cams:
        for _ in range(3):  # the last two launches of each camera run an order built for it
            img, st = gpu_ctx.render(c, 6, precision="f32")
        ordered.append((img, st))
    monkeypatch.setenv("RTC_DEBUG", "tile_order=0")
    with rtc.Context(0) as raster_ctx:
        raster_ctx.upload(scene)
        for c, (img, st) in zip(cams, ordered):
            ref, sr = raster_ctx.render(c, 6, precision="f32")
            assert np.array_equal(img, ref) and _counts(st) == _counts(sr)
