// shape_identity.hpp — value equality of flattened shapes, as the reference
// compares them.
//
// The reference's containers walk finds a shape in its list by VALUE:
// `shapes.iter().position(|shape| *shape == intersection.shape)`
// (composites/intersection.rs:47), where `dyn Shape` equality is `dyn_eq`
// (shapes/shape.rs:34-38, dyn_partial_eq.rs:9-17): same concrete type and
// #[derive(PartialEq)] over every field — the material (material.rs:8,
// including its Option<Arc<dyn Pattern>>, pattern.rs:17-21 and
// complex_pattern.rs:53-60), the inverse transform (matrix.rs:7) and the
// kind's own fields (cylinder.rs:9-15, cone.rs, triangle.rs:9-18).  Two
// value-equal shapes therefore toggle ONE container entry between them.
//
// shape_classes() gives every shape the world index of the first shape it
// equals (its identity class); rt_scene_upload keeps the members of a class
// adjacent in the device table so the kernels' walk can aggregate per class.
// Every comparison is f64 `==` (so -0 == +0 and NaN != NaN, as derive does).
#pragma once

#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "../../include/rtc.h"

namespace rtc {
namespace ident {

inline bool reals_eq(const double* a, const double* b, int n) {
    for (int i = 0; i < n; ++i)
        if (!(a[i] == b[i])) return false;
    return true;
}

// Arc<dyn Pattern> equality by value; `depth` bounds cyclic ComplexPattern
// index graphs (the reference's Arc graph cannot be cyclic).
inline bool pattern_eq(const rt_pattern_desc* P, int a, int b, int depth = 0) {
    if (a == b) return true;
    if (a < 0 || b < 0 || depth > 16) return false;
    const rt_pattern_desc &x = P[a], &y = P[b];
    if (x.kind != y.kind || !reals_eq(x.inverse, y.inverse, 16)) return false;
    if (x.kind == RT_PATTERN_COMPLEX)
        return pattern_eq(P, x.sub_a, y.sub_a, depth + 1) && pattern_eq(P, x.sub_b, y.sub_b, depth + 1);
    if (x.kind == RT_PATTERN_TEST) return true;  // pattern.rs:29-32: the transform only
    return reals_eq(x.color_a, y.color_a, 3) && reals_eq(x.color_b, y.color_b, 3);
}

// material.rs:8-20 #[derive(PartialEq)]
inline bool material_eq(const rt_material_desc* M, const rt_pattern_desc* P, int a, int b) {
    if (a == b) return true;
    const rt_material_desc &m = M[a], &n = M[b];
    return reals_eq(m.color, n.color, 3) && m.ambient == n.ambient && m.diffuse == n.diffuse &&
           m.specular == n.specular && m.shininess == n.shininess && m.reflectiveness == n.reflectiveness &&
           m.transparency == n.transparency && m.refractive_index == n.refractive_index &&
           (m.casts_shadow != 0) == (n.casts_shadow != 0) && pattern_eq(P, m.pattern, n.pattern);
}

// dyn Shape equality (shape.rs:34-38): same kind, then the derived field-wise
// equality of that kind.  A triangle's vertex_2/vertex_3 are not in the
// descriptor; they are compared through vertex_1 + edges.
inline bool shape_eq(const rt_shape_desc* S, const rt_material_desc* M, const rt_pattern_desc* P, uint32_t a,
                     uint32_t b) {
    if (a == b) return true;
    const rt_shape_desc &x = S[a], &y = S[b];
    if (x.kind != y.kind || !reals_eq(x.inverse, y.inverse, 16)) return false;
    if (x.kind == RT_SHAPE_CYLINDER || x.kind == RT_SHAPE_CONE)
        if (!(x.minimum == y.minimum && x.maximum == y.maximum && (x.closed != 0) == (y.closed != 0))) return false;
    if (x.kind == RT_SHAPE_TRIANGLE)
        if (!reals_eq(x.vertex_1, y.vertex_1, 3) || !reals_eq(x.edge_1, y.edge_1, 3) ||
            !reals_eq(x.edge_2, y.edge_2, 3) || !reals_eq(x.normal, y.normal, 3))
            return false;
    return material_eq(M, P, x.material, y.material);
}

// Hash consistent with shape_eq's geometry part (-0 and +0 hash alike);
// materials are compared exactly within a bucket.
inline uint64_t geometry_hash(const rt_shape_desc& s) {
    uint64_t h = 1469598103934665603ull ^ (uint64_t)(uint32_t)s.kind;
    auto mix = [&h](double v) {
        if (v == 0.0) v = 0.0;  // -0 == +0
        uint64_t b;
        std::memcpy(&b, &v, sizeof b);
        h = (h ^ b) * 1099511628211ull;
        h ^= h >> 29;
    };
    for (double v : s.inverse) mix(v);
    if (s.kind == RT_SHAPE_CYLINDER || s.kind == RT_SHAPE_CONE) {
        mix(s.minimum);
        mix(s.maximum);
    }
    return h;
}

// cls[i] = the smallest world index j with shape j == shape i (cls[i] == i
// for a shape equal to no earlier one).  Returns the number of shapes that
// equal an earlier one.
inline uint32_t shape_classes(const rt_shape_desc* S, uint32_t n, const rt_material_desc* M,
                              const rt_pattern_desc* P, std::vector<uint32_t>& cls) {
    cls.resize(n);
    std::unordered_map<uint64_t, std::vector<uint32_t>> buckets;  // hash -> class representatives
    uint32_t dups = 0;
    for (uint32_t i = 0; i < n; ++i) {
        cls[i] = i;
        auto& reps = buckets[geometry_hash(S[i])];
        for (uint32_t r : reps)
            if (shape_eq(S, M, P, r, i)) {
                cls[i] = r;
                ++dups;
                break;
            }
        if (cls[i] == i) reps.push_back(i);
    }
    return dups;
}

}  // namespace ident
}  // namespace rtc
