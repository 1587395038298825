"""CPU checks of the shadow any-hit's wave skips for cubes (rtc_kernels.hip
any_hit), on the kernel's own slab arithmetic (entries(),
cube branch: cube.rs:22-43, 65-85 with the f32 reciprocal) in f32 and f64:

* face separation: both ends of the segment point -> light beyond the same
  face plane of [-1, 1]^3 by 1e-5 (1 + |x|);
* inside: the light 1e-4 inside every face and the point strictly inside.

A lane the kernel skips must be one whose slab test reports no entry with
0 <= t < distance (is_in_shadow, world.rs:98-112), so the skips are exact.
Segments are drawn around cubes of mixed scale, rotation and translation,
with ends placed on, just inside and just outside the faces.
"""
import numpy as np
import pytest


def _transform(rng, dt):
    s = rng.uniform(0.05, 20.0, 3)
    a = rng.uniform(0, 2 * np.pi)
    c, si = np.cos(a), np.sin(a)
    rot = np.array([[c, 0, si], [0, 1, 0], [-si, 0, c]])
    m = rot @ np.diag(s)
    t = rng.uniform(-30, 30, 3)
    inv = np.linalg.inv(m)
    return m, t, inv.astype(dt), (-inv @ t).astype(dt)


def _slab_blocked(o, d, dist, dt):
    """The kernel's cube entries and Blocker test, lane-wise."""
    one, eps, kmax = dt(1), dt(8e-8), np.finfo(dt).max
    tmin = np.full(o.shape[0], -kmax, dt)
    tmax = np.full(o.shape[0], kmax, dt)
    with np.errstate(all="ignore"):
        for a in range(3):
            org, dr = o[:, a], d[:, a]
            nmin, nmax = (-one - org).astype(dt), (one - org).astype(dt)
            steep = np.abs(dr) >= eps
            r = np.where(steep, (one / dr).astype(dt), kmax).astype(dt)
            lo, hi = (nmin * r).astype(dt), (nmax * r).astype(dt)
            lo, hi = np.minimum(lo, hi), np.maximum(lo, hi)
            tmin, tmax = np.maximum(tmin, lo), np.minimum(tmax, hi)
    v = (tmin < tmax) & (tmax > 0)
    hit = lambda t: v & (t >= 0) & (t < dist)  # noqa: E731
    return hit(tmin) | hit(tmax)


def _skips(po, pl, dt):
    one = dt(1)
    lim = lambda x: one + dt(1e-5) * (one + np.abs(x))  # noqa: E731
    la, lb = lim(po), lim(pl)
    out = ((po > la) & (pl > lb)) | ((po < -la) & (pl < -lb))
    clear = out.any(axis=1)
    k_in = dt(1 - 1e-4)
    light_in = (np.abs(pl) < k_in).all(axis=1)
    inside = light_in & (np.abs(po) < one).all(axis=1)
    return clear, inside


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_cube_shadow_skips_are_exact(dt):
    rng = np.random.default_rng(7)
    n_sep = n_in = 0
    for _ in range(200):
        m, t, inv, tinv = _transform(rng, dt)
        n = 2000
        # ends in object space near the faces (on, just in/out) or anywhere
        def ends():
            u = np.where(rng.random((n, 1)) < 0.5, rng.uniform(-3, 3, (n, 3)), rng.uniform(-1, 1, (n, 3)))
            face = rng.integers(0, 3, n)
            side = rng.choice([-1.0, 1.0], n)
            off = rng.choice([0.0, 1e-7, -1e-7, 1e-5, -1e-5, 1e-3, -1e-3, 0.3, -0.3], n)
            near = rng.random(n) < 0.6
            u[near, face[near]] = side[near] * (1 + off[near])
            return u
        po_true, pl_true = ends(), ends()
        p = (po_true @ m.T + t).astype(dt)
        light = (pl_true @ m.T + t).astype(dt)
        v = (light - p).astype(dt)
        dist = np.sqrt((v * v).sum(axis=1)).astype(dt)
        ok = dist > 0
        p, light, v, dist = p[ok], light[ok], v[ok], dist[ok]
        d = (v / dist[:, None]).astype(dt)
        po = (p @ inv.T + tinv).astype(dt)
        pl = (light @ inv.T + tinv).astype(dt)
        ld = (d @ inv.T).astype(dt)
        clear, inside = _skips(po, pl, dt)
        blocked = _slab_blocked(po, ld, dist, dt)
        assert not (clear & blocked).any(), "face separation skipped a blocking cube"
        assert not (inside & blocked).any(), "inside test skipped a blocking cube"
        n_sep += int(clear.sum())
        n_in += int(inside.sum())
    assert n_sep > 10000 and n_in > 1000  # both skips were exercised


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_plane_shadow_side_skip_is_exact(dt):
    """The plane skip (any_hit, K == plane): the point and the light on the same
    side of the plane (object y of one sign) with |y_point| <= 1e4 |y_light|.
    The kernel's plane entry is t = -o.y / d.y (plane.rs:42-48; f32 through the
    reciprocal), valid for |d.y| >= EPSILON; a skipped lane must have no entry
    with 0 <= t < distance."""
    rng = np.random.default_rng(11)
    n_skip = 0
    eps = dt(8e-8)
    for _ in range(200):
        m, t, inv, tinv = _transform(rng, dt)
        n = 2000
        po_true = rng.uniform(-50, 50, (n, 3))
        pl_true = rng.uniform(-50, 50, (n, 3))
        near = rng.random(n) < 0.5
        po_true[near, 1] = rng.choice([1e-6, -1e-6, 1e-3, -1e-3, 1e-5, -1e-5], int(near.sum()))
        lnear = rng.random(n) < 0.3  # lights just off the plane (the ratio cap's case)
        pl_true[lnear, 1] = rng.choice([1e-9, -1e-9, 1e-7, -1e-7, 1e-6, -1e-6], int(lnear.sum()))
        p = (po_true @ m.T + t).astype(dt)
        light = (pl_true @ m.T + t).astype(dt)
        v = (light - p).astype(dt)
        dist = np.sqrt((v * v).sum(axis=1)).astype(dt)
        ok = dist > 0
        p, v, dist, light = p[ok], v[ok], dist[ok], light[ok]
        d = (v / dist[:, None]).astype(dt)
        oy = (p @ inv.T + tinv).astype(dt)[:, 1]
        ly = (light @ inv.T + tinv).astype(dt)[:, 1]
        dy = (d @ inv.T).astype(dt)[:, 1]
        skip = (oy * ly > 0) & (np.abs(oy) <= dt(1e4) * np.abs(ly))
        with np.errstate(all="ignore"):
            tt = (-oy * (dt(1) / dy).astype(dt)).astype(dt)
        blocked = (np.abs(dy) >= eps) & (tt >= 0) & (tt < dist)
        assert not (skip & blocked).any(), "plane side test skipped a blocking plane"
        n_skip += int(skip.sum())
    assert n_skip > 100000
