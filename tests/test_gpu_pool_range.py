"""The ray pool's fixed-point pixel sums and worlds of unbounded colour.

The pool kernel sums a pixel's tree of contributions in int32 (f32) or int64
(f64) fixed point, scaled by a bound on the world's brightest pixel
(rtc_host.cpp scene_brightness / acc_shift_f32).  A TestPattern
(pattern.rs:55-58, reachable through rtc_amd.world.test_pattern()) returns the
pattern-space point as its colour, so its bound comes from the surface's
extent: finite on a sphere, none on a plane.  A bounded world renders and
matches the oracle; an unbounded one is refused with RT_ERR_INVALID rather
than wrapping the sums silently.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _world(W, on_plane, far=0.0):
    tp = W.test_pattern()
    tp.set_transformation(W.scaling(0.5, 0.5, 0.5))
    patterned = W.Material(pattern=tp, ambient=0.3, reflectiveness=0.3)
    floor = W.Material(color=(0.8, 0.8, 0.8), reflectiveness=0.5)
    ball = W.sphere(patterned if not on_plane else W.Material(color=(0.2, 0.4, 0.9), reflectiveness=0.4),
                    W.mat_mul(W.translation(far, 1, far), W.scaling(1, 1, 1)))
    ground = W.plane(floor if not on_plane else patterned)
    return W.World([W.Light((-10, 10, -10))], [ground, ball])


def _camera(W, far=0.0):
    return W.camera(96, 64, 1.0, frm=(far, 1.5, far - 5), to=(far, 1, far), up=(0, 1, 0))


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_test_pattern_on_a_sphere_renders_within_the_bound(gpu_ctx, rtc, oracle, precision):
    from rtc_amd import world as W
    w = _world(W, on_plane=False)
    cam = _camera(W)
    tables = w.tables(cam)
    gpu_ctx.upload(tables)
    img, st = gpu_ctx.render(cam, 6, precision=precision)
    ref, _ = oracle.render(tables, cam, 6, threads=8)
    if precision == "f64":
        assert np.abs(img - ref).max() < 1e-9
    else:
        d = np.abs(oracle.quantize(img).astype(int) - oracle.quantize(ref.astype(np.float64)).astype(int)).max(axis=2)
        assert (d <= 2).mean() >= 0.99


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_test_pattern_on_a_plane_is_refused_by_the_pool(gpu_ctx, rtc, precision):
    from rtc_amd import world as W
    w = _world(W, on_plane=True)
    cam = _camera(W)
    gpu_ctx.upload(w.tables(cam))
    with pytest.raises(rtc.RenderError) as e:
        gpu_ctx.render(cam, 6, precision=precision)
    assert "unbounded" in str(e.value)
    # depth 0 runs the direct kernel, which sums nothing: no bound is needed
    img, _ = gpu_ctx.render(cam, 0, precision=precision)
    assert np.isfinite(img).all()


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test_glass_world_at_the_deepest_supported_depth(gpu_ctx, rtc, oracle, precision):
    """the bound once summed reflectiveness + transparency
    (1.8 for reflect_refract's glass), so (1.8^17 - 1)/0.8 put the f64 bound
    past 2^14 and refused depth 16.  A reflective and transparent material
    mixes its children by Schlick's R and 1 - R (world.rs:59-63), so their
    weight is at most max(r, t) = 0.9 and the frame renders."""
    from conftest import scene_fixture
    scene = scene_fixture("reflect_refract")
    cam = rtc.camera_resize(scene.camera, 96, 64)
    depth = rtc.RT_MAX_SUPPORTED_DEPTH
    gpu_ctx.upload(scene)
    img, st = gpu_ctx.render(cam, depth, precision=precision)
    ref, ref_st = oracle.render(scene, cam, depth, threads=8)
    for k in ("primary", "shadow", "reflect", "refract"):
        assert st[k] == ref_st[k] or precision == "f32", (k, st[k], ref_st[k])
    if precision == "f64":
        assert np.abs(img - ref).max() < 1e-9
    else:
        d = np.abs(oracle.quantize(img).astype(int) - oracle.quantize(ref.astype(np.float64)).astype(int)).max(axis=2)
        assert (d <= 2).mean() >= 0.97
