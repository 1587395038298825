"""The defines a per-scene build adds by kernel kind (csrc/jit_options.hpp,
used by rtc_jit.cpp make_request), checked on the CPU: the direct kernel keeps
its shape records as constants and fences every third shape, the pool kernel
takes records from LDS, and only RT_FLAG_NO_SKIPS builds drop the skips.
Round 5 ran for a while with every build but the no-skips ones compiled
without records (an `else` bound to a newly inserted `if`): the direct kernel
was 13 % slower (three_sphere 1080p 15.5 -> 17.7 us, same box) and no test
saw it, since records change speed only.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "ray-tracer-challenge-rs_amd", "csrc")

PROG = r"""
#include <cstdio>
#include "jit_options.hpp"
int main() {
    for (int pool = 0; pool < 2; ++pool)
        for (int ns = 0; ns < 2; ++ns) {
            std::printf("%d %d", pool, ns);
            for (const auto& d : rtc::jit_kind_defines(pool, ns)) std::printf(" %s", d.c_str());
            std::printf("\n");
        }
    std::printf("w7");  // the pool kernel's 7-wave attempt (rtc_jit.cpp jit_function)
    for (const auto& d : rtc::jit_kind_defines(true, false, 7)) std::printf(" %s", d.c_str());
    std::printf("\nw7direct");
    for (const auto& d : rtc::jit_kind_defines(false, false, 7)) std::printf(" %s", d.c_str());
    std::printf("\n");
}
"""


def test_kind_defines(tmp_path):
    src = tmp_path / "opts.cpp"
    src.write_text(PROG)
    exe = tmp_path / "opts"
    subprocess.run(["g++", "-std=c++17", "-O0", "-I", CSRC, "-o", str(exe), str(src)], check=True)
    rows, extra = {}, {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        if line.startswith("w7"):
            tag, *defs = line.split()
            extra[tag] = set(defs)
            continue
        pool, ns, *defs = line.split()
        rows[(pool == "1", ns == "1")] = set(defs)
    assert "-DRTC_POOL_WAVES=7" in extra["w7"] and "-DRTC_JIT_NO_RECORDS" in extra["w7"]
    assert not any(d.startswith("-DRTC_POOL_WAVES") for d in extra["w7direct"])  # the direct kernel ignores it
    for ns in (False, True):
        direct, pool = rows[(False, ns)], rows[(True, ns)]
        assert "-DRTC_JIT_NO_RECORDS" not in direct and "-DRTC_JIT_FENCE_EVERY=3" in direct
        assert "-DRTC_JIT_FENCE_MIN_SHAPES=9" in direct
        assert "-DRTC_JIT_NO_RECORDS" in pool and not any(d.startswith("-DRTC_JIT_FENCE_EVERY") for d in pool)
        assert ("-DRTC_NO_SKIPS" in direct) == ns and ("-DRTC_NO_SKIPS" in pool) == ns
