"""CPU checks of the pool kernel's index arithmetic (no GPU).

* tests/index_math.cpp, built with g++ against rtc_internal.hpp (the header
  the kernels include): work-item encode/decode (packed only in tile-ordered
  launches, plain tiles of any size in raster ones: ADVICE r3), the threads a
  split part seeds, spill record addressing, the row-block shard maps.
* The LIFO bound the pool's capacity rests on (rtc_host.cpp pool_capacity:
  kBlock + depth x batch): a model of trace_pool's generation loop
  (rtc_kernels.hip: pop the top min(size, 256) rays, push each popped ray's
  0-2 children with remaining - 1, in any order) never holds more.  This is
  the reference's recursion (world.rs:114-157: a shaded hit spawns at most a
  reflected and a refracted ray while remaining > 0) run LIFO.
"""
import os
import random
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BLOCK = 256


def test_index_math_cpp(tmp_path):
    exe = tmp_path / "index_math"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-o", str(exe), os.path.join(HERE, "index_math.cpp")],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    lines = out.stdout.split()
    assert out.returncode == 0 and lines[-1] == "ok", out.stdout + out.stderr
    # kErrBitsAll lists every kErr* constant of the header
    import re
    hdr = open(os.path.join(HERE, "..", "ray-tracer-challenge-rs_amd", "csrc", "rtc_internal.hpp")).read()
    declared = re.findall(r"constexpr int32_t (kErr\w+) = ", hdr)
    assert f"errbits {len(declared)}" in out.stdout, (declared, out.stdout)


def _pool_peak(depth, seeds, rng, children):
    stack = [depth] * seeds
    peak = len(stack)
    while stack:
        k = min(len(stack), BLOCK)
        popped = stack[-k:]
        del stack[-k:]
        kids = []
        for rem in popped:
            if rem > 0:
                kids += [rem - 1] * children(rng)
        rng.shuffle(kids)  # wave_reserve order is arbitrary
        stack += kids
        peak = max(peak, len(stack))
    return peak


@pytest.mark.parametrize("policy", ["both", "random", "mostly_both"])
def test_lifo_pool_bound(policy):
    children = {"both": lambda r: 2, "random": lambda r: r.choice((0, 1, 2)),
                "mostly_both": lambda r: r.choice((0, 1, 2, 2, 2))}[policy]
    rng = random.Random(7)
    for depth in range(0, 9):
        cap = BLOCK + depth * BLOCK
        for seeds in (1, 16, 32, 64, 128, 200, 256):  # split parts seed 256 >> l threads
            for _ in range(1 if policy == "both" else 12):
                peak = _pool_peak(depth, seeds, rng, children)
                assert peak <= cap, (depth, seeds, peak, cap)
                if policy == "both" and seeds == BLOCK:
                    assert peak == cap  # the bound is tight: every ray spawning both children
