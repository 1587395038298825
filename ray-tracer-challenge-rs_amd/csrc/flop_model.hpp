// flop_model.hpp — the algorithmic-FLOP convention of SURVEY.md §8(d), frozen
// in one place.  `roofline.achieved` (bench.py) divides these FLOPs by the
// measured kernel time.
//
// Convention: +, -, x, /, sqrt, min, max = 1 flop; FMA = 2; compares, abs,
// negation and casts = 0; powf = 1.  EVERY traced ray (primary, shadow,
// reflect, refract) is charged brute force over ALL shapes, as the reference
// does (world.rs:31-33, 107): the kernel gets no credit for early exits.
//
//   term                                   flops  derivation (reference file:line)
//   ray -> object affine transform            33  ray.rs:45-49
//   sphere test                          33 + 27  sphere.rs:42-46, utils.rs:48-56
//   plane test                           33 +  1  plane.rs:46
//   cube test                            33 + 18  cube.rs:25-36, 70-77
//   cylinder open / closed          33 + 25 / 43  cylinder.rs:82-105 (+ caps 34-58)
//   cone open / closed              33 + 30 / 50  cone.rs:82-108 (+ caps 34-58)
//   triangle test                        33 + 44  triangle.rs:40-53
//   per shaded hit (prepare)                  79  intersection.rs:22-31, shape.rs:22-27, computed_hit.rs:33-34
//   per light per shaded hit                  82  world.rs:104-106 (18) + material.rs:92-113 (61) + 3
//     ... if the material is patterned       +40  pattern.rs:11-13
//   refracted_color past its guards           23  world.rs:140-151
//   schlicks_approximation                    22  computed_hit.rs:51-67
//   per shaded hit (combine)                  12  world.rs:59-66
#pragma once

#include <cstdint>

#include "../../include/rtc.h"

namespace rtc {

struct FlopScene {
    double per_ray = 0;  // Σ over shapes of the per-shape test (incl. the transform)
    uint32_t n_lights = 0;
};

inline double shape_test_flops(int kind, bool closed) {
    switch (kind) {
        case RT_SHAPE_SPHERE: return 60;
        case RT_SHAPE_PLANE: return 34;
        case RT_SHAPE_CUBE: return 51;
        case RT_SHAPE_CYLINDER: return closed ? 76 : 58;
        case RT_SHAPE_CONE: return closed ? 83 : 63;
        default: return 77;  // triangle
    }
}

// FLOPs/frame = Σ_rays Σ_shapes F + Σ_shaded (79 + Σ_L (82 + 40·pat) + 23·[refract] + 22·[schlick] + 12)
inline double algorithmic_flops(const FlopScene& s, const rt_stats& k) {
    const double rays = (double)k.primary + (double)k.reflect + (double)k.refract + (double)k.shadow;
    return rays * s.per_ray + (double)k.shaded * (79.0 + 12.0) + (double)k.shadow * 82.0 +
           (double)k.lit_patterned * 40.0 + (double)k.refract_evals * 23.0 + (double)k.schlick_evals * 22.0;
}

}  // namespace rtc
