"""Value identity of shapes on the GPU.

The reference's containers walk removes a shape from its list when it finds
an entry of a shape EQUAL BY VALUE to it (`shapes.iter().position(|shape|
*shape == intersection.shape)`, composites/intersection.rs:47; `dyn Shape`
equality is dyn_eq over #[derive(PartialEq)], shapes/shape.rs:34-38).  Two
value-equal overlapping glass spheres therefore give different n1/n2 than
two distinct ones.  The device groups value-equal shapes into one identity
class (rt_scene_upload, csrc/shape_identity.hpp) and its walk toggles one
entry per class; the oracle compares shapes by value (rtc_oracle.hpp
shape_eq), so the two must agree to 1e-9 in f64 with identical counters.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ABS64 = 1e-9


def _counts(st):
    return {k: st[k] for k in ("primary", "shadow", "reflect", "refract", "shaded", "lit_patterned",
                               "refract_evals", "schlick_evals")}


def _dup_world(perturb=0.0):
    from test_identity import dup_world
    return dup_world(perturb)


def _cam():
    from rtc_amd import world as W
    return W.camera(96, 72, 0.9, (0, 0.6, -5), (0.2, 0, 0), (0, 1, 0))


def _rays(n=4096, seed=5):
    rng = np.random.default_rng(seed)
    o = np.tile([0.0, 0.6, -5.0], (n, 1)) + rng.normal(scale=0.05, size=(n, 3))
    tgt = np.array([0.4, 0.2, -1.6]) + rng.normal(scale=0.45, size=(n, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], axis=1)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_value_equal_shapes_render_like_the_oracle(gpu_ctx, oracle, precision):
    tables = _dup_world()
    cam = _cam()
    gpu_ctx.upload(tables)
    img, st = gpu_ctx.render(cam, 6, precision=precision)
    ref, rst = oracle.render(tables, cam, 6, threads=8)
    if precision == "f64":
        assert np.abs(img - ref).max() < ABS64
        assert _counts(st) == _counts(rst)
    else:
        d = np.abs(oracle.quantize(img).astype(int) - oracle.quantize(ref).astype(int)).max(axis=2)
        assert (d <= 2).mean() >= 0.99


def test_value_equal_shapes_color_at(gpu_ctx, oracle):
    tables = _dup_world()
    rays = _rays()
    gpu_ctx.upload(tables)
    got, st = gpu_ctx.color_at(rays, depth=6, precision="f64")
    orc, ost = oracle.color_at(tables, rays, depth=6)
    assert np.abs(got - orc).max() < ABS64
    assert _counts(st) == _counts(ost)


def test_unequal_pair_renders_like_the_oracle(gpu_ctx, oracle):
    """The same pair made unequal (ambient off by 1e-15): two classes, which
    the oracle renders differently through the spheres (tests/test_identity.py)."""
    from test_identity import dup_world
    cam = _cam()
    tables = dup_world(perturb=1e-15)
    ne, nst = oracle.render(tables, cam, 6, threads=8)
    gpu_ctx.upload(tables)
    img, st = gpu_ctx.render(cam, 6, precision="f64")
    assert np.abs(img - ne).max() < ABS64
    assert _counts(st) == _counts(nst)
