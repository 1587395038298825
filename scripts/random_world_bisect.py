"""Diagnostic: localise an f64 GPU/oracle difference in a random world of
tests/test_gpu_random_worlds.py.  For each seed given: the differing pixels,
then the same count with each shape removed in turn, and with each
material feature switched off, so the shape and feature behind it show."""
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("ray-tracer-challenge-rs_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import pyoracle  # noqa: E402
import rtc_amd  # noqa: E402
from rtc_amd import world as W  # noqa: E402
import test_gpu_random_worlds as T  # noqa: E402

captured = {}
_World = W.World


class _Capture(_World):
    def tables(self, camera=None):
        captured["world"] = self
        return _World.tables(self, camera)


def bad_pixels(ctx, world, cam, depth, flags=0):
    tables = world.tables()
    ctx.upload(tables)
    ref, _ = pyoracle.render(tables, cam, depth, threads=8)
    img, _ = ctx.render(cam, depth, precision="f64", flags=flags)
    d = np.abs(img - ref).max(axis=2)
    ys, xs = np.nonzero(d > 1e-9)
    return len(ys), (float(d.max()) if len(ys) else 0.0), list(zip(xs[:4].tolist(), ys[:4].tolist()))


def main():
    W.World = _Capture
    with rtc_amd.Context(0) as ctx:
        for seed in [int(a) for a in sys.argv[1:]] or [5]:
            _, cam, depth = T._random_world(seed)
            world = captured["world"]
            n, mx, where = bad_pixels(ctx, world, cam, depth)
            print(f"seed {seed} depth {depth}: {n} pixels differ, max {mx:.3g}, e.g. {where}", flush=True)
            if not n:
                continue
            print(f"  RT_FLAG_NO_SKIPS: {bad_pixels(ctx, world, cam, depth, rtc_amd.RT_FLAG_NO_SKIPS)[:2]}  "
                  f"(RTC_DEBUG={os.environ.get('RTC_DEBUG', '')})", flush=True)
            if os.environ.get("RTC_DEBUG"):
                continue
            for i, s in enumerate(world.shapes):
                w2 = copy.deepcopy(world)
                del w2.shapes[i]
                print(f"  without shape {i} ({s.kind}): {bad_pixels(ctx, w2, cam, depth)[:2]}", flush=True)
            for feat in ("pattern", "reflectiveness", "transparency", "casts_shadow"):
                w2 = copy.deepcopy(world)
                for s in w2.shapes:
                    if feat == "pattern":
                        s.material.pattern = None
                    elif feat == "casts_shadow":
                        s.material.casts_shadow = True
                    else:
                        setattr(s.material, feat, 0.0)
                print(f"  without {feat}: {bad_pixels(ctx, w2, cam, depth)[:2]}", flush=True)
            for d2 in range(depth):
                print(f"  depth {d2}: {bad_pixels(ctx, world, cam, d2)[:2]}", flush=True)


if __name__ == "__main__":
    main()
