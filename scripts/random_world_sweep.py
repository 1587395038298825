"""GPU sweep (not a test: too long for the suite): the random worlds of
tests/test_gpu_random_worlds.py at 480x360 through the per-scene kernels,
against the generic kernel, the per-scene kernel with the cull off
(RTC_DEBUG=cull=0) and with RT_FLAG_NO_SKIPS: every f32 frame bit for bit.
One JSON line per seed."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("ray-tracer-challenge-rs_amd", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import rtc_amd  # noqa: E402
import test_gpu_random_worlds as T  # noqa: E402


def frame(ctx, tables, cam, depth, flags=0):
    ctx.upload(tables)
    img, st = ctx.render(cam, depth, precision="f32", flags=flags)
    return img, T._counts(st)


def main():
    seeds = [int(a) for a in sys.argv[1:]] or list(range(32))
    bad = 0
    for seed in seeds:
        for plain in (False, True):
            tables, cam, depth = T._random_world(seed, plain=plain, allow_dup=False)
            cam = rtc_amd.camera_resize(cam, 480, 360)
            os.environ.pop("RTC_DEBUG", None)
            with rtc_amd.Context(0) as gen, rtc_amd.Context(0) as jit:
                gen.set_jit(rtc_amd.RT_JIT_OFF)
                jit.set_jit(rtc_amd.RT_JIT_SYNC)
                a, ca = frame(gen, tables, cam, depth)
                b, cb = frame(jit, tables, cam, depth)
                used = jit.jit_status()["used"]
                c, cc = frame(jit, tables, cam, depth, rtc_amd.RT_FLAG_NO_SKIPS)
            os.environ["RTC_DEBUG"] = "cull=0"
            with rtc_amd.Context(0) as nocull:
                nocull.set_jit(rtc_amd.RT_JIT_SYNC)
                d, cd = frame(nocull, tables, cam, depth)
            os.environ.pop("RTC_DEBUG", None)
            diff = {k: int((a != x).any(axis=2).sum()) for k, x in (("jit", b), ("jit_no_skips", c), ("jit_no_cull", d))}
            same_counts = ca == cb == cc == cd
            ok = not any(diff.values()) and same_counts
            bad += not ok
            print(json.dumps({"seed": seed, "plain": plain, "depth": depth, "jit_used": used, "px_differ": diff,
                              "counters_equal": same_counts, "ok": ok}), flush=True)
    print(json.dumps({"worlds": 2 * len(seeds), "failed": bad}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
