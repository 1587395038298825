"""Seeded random worlds: the HIP path against the f64 oracle beyond the
reference's scenes.

The reference scenes hold no cone or triangle, no sheared or rotated
cylinder, no value-identical pair of shapes and no light count above two.
Each seed here draws a world with every shape kind (world.rs:25-35 with
shapes/*.rs), random transforms with rotation, non-uniform scale and shear
(shape.rs:22-27), random Phong materials with reflection, refraction and
Schlick mixing (world.rs:38-67, 114-157), every pattern kind but the test
pattern (pattern.rs), shapes that cast no shadow (world.rs:108-111),
sometimes a value-identical copy of a shape (intersection.rs:47), one to
three lights, and a depth of 0 to 6.  A small frame of it is rendered in
f64 (every pixel within 1e-9 of the oracle, every ray counter equal) and in
f32 (pixels within 2/255 after canvas.rs:117-123's quantization, a floor set
from the observed agreement of these seeds with a margin).
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ABS64 = 1e-9
F32_PIX_FRAC = 0.99  # observed minimum over the 48 seeds: 0.9958 (round 6)
SEEDS = list(range(48))


def rtc_amd_error():
    import rtc_amd
    return rtc_amd.RenderError


def depth_has_pool(tables):
    """Some material reflective or transparent (the pool kernel's worlds)."""
    return any(m.reflectiveness != 0 or m.transparency != 0 for m in tables.materials)


def _counts(st):
    return {k: st[k] for k in ("primary", "shadow", "reflect", "refract", "shaded", "lit_patterned",
                               "refract_evals", "schlick_evals")}


def _random_world(seed, plain=False, allow_dup=True, light_scale=1.0):
    """(tables, camera, depth) of seed's world.  plain: no reflective or
    transparent material (the direct kernel's worlds); allow_dup=False: no
    value-identical copy; light_scale: brighter lights (the f32 pixel sums'
    fixed-point scale follows the world's brightness bound).  None of them
    changes the draws of the other parts."""
    from rtc_amd import world as W
    rng = np.random.default_rng(seed)

    def u(lo, hi):
        return float(rng.uniform(lo, hi))

    def color():
        return (u(0, 1), u(0, 1), u(0, 1))

    def transform(scale_lo=0.3, scale_hi=1.4):
        m = W.translation(u(-3, 3), u(0, 2.5), u(-3, 3))
        m = W.mat_mul(m, W.rotation_y(u(0, 2 * math.pi)))
        if rng.random() < 0.6:
            m = W.mat_mul(m, W.rotation_x(u(-1, 1)))
            m = W.mat_mul(m, W.rotation_z(u(-1, 1)))
        if rng.random() < 0.25:
            m = W.mat_mul(m, W.shearing(*[u(-0.3, 0.3) for _ in range(6)]))
        s = u(scale_lo, scale_hi)
        if rng.random() < 0.5:
            return W.mat_mul(m, W.scaling(s, s, s))
        return W.mat_mul(m, W.scaling(s, u(scale_lo, scale_hi), u(scale_lo, scale_hi)))

    def pattern():
        kind = int(rng.integers(0, 5))
        if kind == 4:
            p = W.complex_pattern(W.stripe_pattern(color(), color()), W.checker_pattern(color(), color()))
        else:
            p = (W.stripe_pattern, W.gradient_pattern, W.ring_pattern, W.checker_pattern)[kind](color(), color())
        if rng.random() < 0.5:
            p.set_transformation(W.mat_mul(W.rotation_y(u(0, 3)), W.scaling(u(0.2, 1), u(0.2, 1), u(0.2, 1))))
        return p

    def material():
        m = W.Material(color=color(), ambient=u(0, 0.3), diffuse=u(0.3, 1), specular=u(0, 1),
                       shininess=u(5, 300), casts_shadow=bool(rng.random() < 0.85))
        if rng.random() < 0.3:
            m.pattern = pattern()
        if rng.random() < 0.35:
            m.reflectiveness = u(0.1, 0.9)
        if rng.random() < 0.3:
            m.transparency = u(0.2, 1.0)
            m.refractive_index = u(1.0, 2.0)
        return m

    shapes = [W.plane(material(), W.translation(0, u(-1.5, -0.5), 0))]
    if rng.random() < 0.3:  # a back wall
        shapes.append(W.plane(material(), W.mat_mul(W.translation(0, 0, 6), W.rotation_x(math.pi / 2))))
    for _ in range(int(rng.integers(3, 9))):
        kind = int(rng.integers(0, 5))
        if kind == 0:
            shapes.append(W.sphere(material(), transform()))
        elif kind == 1:
            shapes.append(W.cube(material(), transform(0.2, 0.9)))
        elif kind == 2:
            lo = u(-1, 0.5)
            bounded = rng.random() < 0.8
            shapes.append(W.cylinder(lo if bounded else -W.F64_MAX, lo + u(0.2, 2) if bounded else W.F64_MAX,
                                     bool(rng.random() < 0.6), material(), transform(0.2, 0.9)))
        elif kind == 3:
            lo = u(-1.5, -0.2)
            shapes.append(W.cone(lo, u(-0.1, 1.0) if rng.random() < 0.5 else 0.0, bool(rng.random() < 0.6),
                                 material(), transform(0.3, 1.0)))
        else:
            c = (u(-3, 3), u(0, 2), u(-3, 3))
            pts = [tuple(c[q] + u(-1.2, 1.2) for q in range(3)) for _ in range(3)]
            shapes.append(W.triangle(*pts, material()))
    if rng.random() < 0.25:  # a value-identical copy (the containers walk's identity classes)
        import copy
        at, src = int(rng.integers(0, len(shapes))), int(rng.integers(1, len(shapes)))
        if allow_dup:
            shapes.insert(at, copy.deepcopy(shapes[src]))
    if plain:
        for sh in shapes:
            sh.material.reflectiveness = sh.material.transparency = 0.0
    lights = [W.Light((u(-8, 8), u(4, 10), u(-10, -2)),
                      (light_scale * u(0.3, 1), light_scale * u(0.3, 1), light_scale * u(0.3, 1)))
              for _ in range(int(rng.integers(1, 4)))]
    eye = (u(-4, 4), u(1.5, 4), u(-9, -6))
    cam = W.camera(96, 72, u(0.6, 1.2), eye, (0, 0.5, 0), (0, 1, 0))
    return W.World(lights, shapes).tables(), cam, int(rng.integers(0, 7))


@pytest.mark.parametrize("seed", SEEDS + [f"{s}x4" for s in range(8)])
def test_random_world_parity(gpu_ctx, oracle, seed):
    """Seeds "<s>x4": the same world with lights four times as bright."""
    if isinstance(seed, str):
        tables, cam, depth = _random_world(int(seed[:-2]), light_scale=4.0)
    else:
        tables, cam, depth = _random_world(seed)
    gpu_ctx.upload(tables)
    ref, rst = oracle.render(tables, cam, depth, threads=8)
    img, st = gpu_ctx.render(cam, depth, precision="f64")
    err = float(np.abs(img - ref).max())
    assert err < ABS64, f"seed {seed}: f64 max |err| {err:.3g}"
    assert _counts(st) == _counts(rst), f"seed {seed}"
    img32, _ = gpu_ctx.render(cam, depth, precision="f32")
    d = np.abs(oracle.quantize(img32).astype(int) - oracle.quantize(ref).astype(int)).max(axis=2)
    agree = float((d <= 2).mean())
    # the next frames are cost-ordered (heavy tiles split, raised priority): the same pixels
    for precision, first in (("f32", img32), ("f64", img)):
        again, _ = gpu_ctx.render(cam, depth, precision=precision)
        assert np.array_equal(again, first), f"seed {seed}: warm {precision} frame differs"
    print(f"seed {seed} depth {depth} shapes {len(tables.shapes)}: f64 {err:.2e}, f32 within 2/255 {agree:.4f}")
    assert agree >= F32_PIX_FRAC, f"seed {seed}: f32 {agree:.4f}"


@pytest.mark.parametrize("plain", [False, True], ids=["pool", "direct"])
@pytest.mark.parametrize("seed", list(range(16)))
def test_random_world_per_scene_kernel_equals_generic(rtc, seed, plain):
    """The per-scene (hipRTC) kernels the bench runs, built for each random
    world (constant shape records, clusters, world-space spheres and cubes,
    the acceleration skips), against the generic f32 kernel: the same
    frame bit for bit and the same counters.  (21 of these 32 builds were
    accepted in round 6; the others were refused for scratch.)"""
    tables, cam, depth = _random_world(seed, plain=plain, allow_dup=False)
    with rtc.Context(0) as gen, rtc.Context(0) as jit:
        gen.set_jit(rtc.RT_JIT_OFF)
        jit.set_jit(rtc.RT_JIT_SYNC)
        gen.upload(tables)
        jit.upload(tables)
        a, sa = gen.render(cam, depth, precision="f32")
        b, sb = jit.render(cam, depth, precision="f32")
        js = jit.jit_status()
        if not js["used"]:
            # a build that spills or loses occupancy is refused (rtc_jit.cpp
            # jit_variant), with its reason in the log, and the frame falls
            # back to the generic kernel (checked below like an accepted one)
            assert "not used" in js["log"] and ("scratch" in js["log"] or "workgroups/CU" in js["log"]), js
        assert np.array_equal(a, b), f"seed {seed}: {int((a != b).any(axis=2).sum())} pixels differ"
        assert _counts(sa) == _counts(sb)


@pytest.mark.parametrize("seed", list(range(16)))
def test_random_world_color_at_random_rays(gpu_ctx, oracle, seed):
    """World::color_at (world.rs:89-93) on 2048 random rays per random world:
    origins anywhere in the scene's box, inside shapes included (the
    containers walk then starts with entries at t < 0), unit directions.
    f64 within 1e-9 of the oracle's color_at, counters equal.  (Non-unit
    directions are refused in worlds with secondary rays, rtc.h rt_color_at:
    the specular term grows as |d|^shininess past the pool's fixed-point
    range.)"""
    tables, _, _ = _random_world(seed)
    rng = np.random.default_rng(1000 + seed)
    n = 2048
    o = rng.uniform([-4, -1.5, -6], [4, 4, 4], size=(n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], axis=1)
    gpu_ctx.upload(tables)
    if depth_has_pool(tables):
        bad = rays.copy()
        bad[7, 3:] *= 1.5
        with pytest.raises(rtc_amd_error(), match="unit length"):
            gpu_ctx.color_at(bad, 6, precision="f64")
    got, st = gpu_ctx.color_at(rays, 6, precision="f64")
    ref, rst = oracle.color_at(tables, rays, 6)
    err = float(np.abs(got - ref).max())
    assert err < ABS64, f"seed {seed}: max |err| {err:.3g} at ray {int(np.abs(got - ref).max(axis=1).argmax())}"
    assert _counts(st) == _counts(rst), f"seed {seed}"


def _many_shapes_world(seed, n):
    """A world of n small shapes (spheres, cubes, closed cylinders, triangles)
    scattered over a floor, a fifth of them reflective or glass: past the
    per-scene builds' record limit (255 shapes) and the LDS world tables."""
    from rtc_amd import world as W
    rng = np.random.default_rng(seed)

    def u(lo, hi):
        return float(rng.uniform(lo, hi))

    shapes = [W.plane(W.Material(color=(0.8, 0.8, 0.7), reflectiveness=0.1), W.translation(0, -0.2, 0))]
    for _ in range(n):
        m = W.Material(color=(u(0, 1), u(0, 1), u(0, 1)), specular=u(0, 1), shininess=u(10, 200))
        r = rng.random()
        if r < 0.1:
            m.reflectiveness = u(0.2, 0.9)
        elif r < 0.2:
            m.transparency, m.refractive_index = u(0.5, 1.0), u(1.1, 1.8)
        s = u(0.05, 0.25)
        t = W.mat_mul(W.translation(u(-6, 6), u(0, 3), u(-4, 8)), W.rotation_y(u(0, 3)))
        k = int(rng.integers(0, 4))
        if k == 0:
            shapes.append(W.sphere(m, W.mat_mul(t, W.scaling(s, s, s))))
        elif k == 1:
            shapes.append(W.cube(m, W.mat_mul(t, W.scaling(s, s, s))))
        elif k == 2:
            shapes.append(W.cylinder(-1, 1, True, m, W.mat_mul(t, W.scaling(s, s, s))))
        else:
            c = (u(-6, 6), u(0, 3), u(-4, 8))
            shapes.append(W.triangle(*[tuple(c[q] + u(-0.3, 0.3) for q in range(3)) for _ in range(3)], m))
    lights = [W.Light((-10, 10, -10)), W.Light((8, 12, -4), (0.4, 0.4, 0.5))]
    cam = W.camera(80, 60, 1.1, (0, 2.5, -9), (0, 1, 2), (0, 1, 0))
    return W.World(lights, shapes).tables(), cam


@pytest.mark.parametrize("n", [300, 1500])
def test_many_shapes_world(gpu_ctx, oracle, rtc, n):
    """Hundreds to thousands of shapes: f64 within 1e-9 of the oracle with
    equal counters, f32 within 2/255, and the per-scene kernels (clusters,
    or the generic tables past 255 shapes) bit-equal to the generic one."""
    tables, cam = _many_shapes_world(n, n)
    gpu_ctx.upload(tables)
    ref, rst = oracle.render(tables, cam, 4, threads=8)
    img, st = gpu_ctx.render(cam, 4, precision="f64")
    assert float(np.abs(img - ref).max()) < ABS64
    assert _counts(st) == _counts(rst)
    img32, s32 = gpu_ctx.render(cam, 4, precision="f32")
    d = np.abs(oracle.quantize(img32).astype(int) - oracle.quantize(ref).astype(int)).max(axis=2)
    assert float((d <= 2).mean()) >= F32_PIX_FRAC
    with rtc.Context(0) as jit:
        jit.set_jit(rtc.RT_JIT_SYNC)
        jit.upload(tables)
        b, sb = jit.render(cam, 4, precision="f32")
        assert np.array_equal(img32, b) and _counts(s32) == _counts(sb), jit.jit_status()


@pytest.mark.parametrize("seed", list(range(24)))
def test_random_world_accelerations_are_exact(gpu_ctx, rtc, monkeypatch, seed):
    """The wave cull and the shadow/exit skips are acceleration only: on every
    random world the f32 and f64 frames with the cull off (RTC_DEBUG=cull=0,
    every shape unbounded) and with RT_FLAG_NO_SKIPS equal the default frame
    bit for bit, counters included.  (An f32 decision flipped on one pixel
    would pass the oracle's 2/255 floor; this catches it.)"""
    tables, cam, depth = _random_world(seed)
    gpu_ctx.upload(tables)
    monkeypatch.setenv("RTC_DEBUG", "cull=0")
    with rtc.Context(0) as nocull:
        nocull.upload(tables)
        for precision in ("f32", "f64"):
            a, sa = gpu_ctx.render(cam, depth, precision=precision)
            b, sb = nocull.render(cam, depth, precision=precision)
            c, sc = gpu_ctx.render(cam, depth, precision=precision, flags=rtc.RT_FLAG_NO_SKIPS)
            assert np.array_equal(a, b), f"seed {seed} {precision}: the cull changed {int((a != b).any(axis=2).sum())} px"
            assert np.array_equal(a, c), f"seed {seed} {precision}: the skips changed {int((a != c).any(axis=2).sum())} px"
            assert _counts(sa) == _counts(sb) == _counts(sc)
