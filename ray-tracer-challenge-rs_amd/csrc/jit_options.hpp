// jit_options.hpp — the defines a per-scene build adds by kernel kind
// (rtc_jit.cpp make_request), kept apart so a CPU test can check them
// (tests/test_jit_options.py): round 5 lost the direct kernel's constant
// records for a while to an `else` that bound to the wrong `if`.
#pragma once
#include <string>
#include <vector>

namespace rtc {

// pool_waves: the pool kernel's waves per SIMD (RTC_POOL_WAVES), 0 = the
// static build's.  rtc_jit.cpp compiles 7 beside the static occupancy and
// keeps the 7-wave build when it spills at most kPool7ScratchMax (round 5,
// same box against 6: table 4K -3.6 %, cover 4K -4.3 %, reflect_refract
// -2.4 %); cylinders' build spills 44 B/lane at 7 and takes the other.
inline std::vector<std::string> jit_kind_defines(bool pool, bool no_skips, int pool_waves = 0) {
    std::vector<std::string> d;
    if (pool && pool_waves > 0) d.push_back("-DRTC_POOL_WAVES=" + std::to_string(pool_waves));
    // The direct kernel fences the ray at every third shape only: the shape
    // tests in between may interleave (more ILP) and still fit 8 waves/SIMD
    // without spilling.  Same-box A/B against a fence per shape: shadow_puppets
    // -3.6 %, three_sphere 4K -2.5 %, 1080p -0.6 %; the pool kernel lost 15 %
    // on cover that way and keeps a fence per shape.  Worlds of at most 8
    // shapes take no fence (round 5, same box: three_sphere 15.48 -> 15.31 us,
    // shadow_puppets 19.69 -> 18.90 us; 36 VGPRs, no spills).
    if (!pool) {
        d.push_back("-DRTC_JIT_FENCE_EVERY=3");
        d.push_back("-DRTC_JIT_FENCE_MIN_SHAPES=9");
    }
    // Shape records as constants (rtc_kernels.hip kJitRecords) pay off in the
    // direct kernel only.  Same-box A/B, two rounds (profiles/ab/r04_ab_builds.log):
    // direct three_sphere 17.0 us with them vs 18.4 us without; pool kernels
    // without them reflect_refract -3.0 %, table -1.2 %, cover -0.6 % (the
    // per-slot branches cost more than the extra LDS pool slots gain).
    if (pool) d.push_back("-DRTC_JIT_NO_RECORDS");
    // RT_FLAG_NO_SKIPS launches (exactness tests) run a build without the skips
    if (no_skips) d.push_back("-DRTC_NO_SKIPS");
    return d;
}

}  // namespace rtc
