// rtc_kernels.hip — the MI355X (gfx950, wave64) render path.
//
// Replaces Camera::render[_parallel] (camera.rs:79-112) and the
// World::color_at -> collect_intersections -> shade_hit recursion
// (world.rs:25-157) with two persistent-threads kernels:
//
//  * trace_direct  — one thread per pixel, no ray pool.  Used when no ray can
//    spawn a child (no material with reflectiveness/transparency != 0, or
//    max_depth == 0): the whole per-pixel tree is one shaded hit plus L shadow
//    rays.  This is three_sphere_scene, the BASELINE metric's config.
//  * trace_pool    — wavefront tracer.  A workgroup owns a 64x4 tile
//    (RT_TILE_W x RT_TILE_H, each wave a 16x4 block of it); the tile's rays
//    live in LDS (SoA) as a LIFO pool.  Each iteration pops up to
//    `pop_batch` rays, traces them one per lane (closest hit, shading, any-hit
//    shadow rays), accumulates weight x surface colour into the tile's pixel
//    accumulators, and pushes the reflection/refraction children, compacted
//    per wave with ballot + mbcnt and ONE LDS atomic per wave.  LIFO popping
//    bounds the pool at tile + depth x pop_batch rays (host sizes it).
//    The recursion is linear in scalar weights (world.rs:54-66, 127, 156), so
//    pixel = sum over tree nodes of (product of weights) x surface colour.
//
// Pool tiles are handed out by 8 per-XCD atomic queues with stealing
// (dynamic load balance over a grid sized to the resident workgroup count),
// heaviest first once a launch has recorded the tiles' costs; direct tiles by
// a static stride over 2.5x the resident grid.  World tables are read
// with wave-uniform scalar loads in per-type loops (rtc_internal.hpp).
//
// Two instantiations: R = float (the throughput path) and R = double (parity:
// the reference's operation order, its FMA sites and EPSILON = 8e-8; the TU
// is compiled with -ffp-contract=off so nothing else is fused).
//
// Precision split: RTC_PRECISION=1 compiles the f32 kernels (and the helper
// kernels), RTC_PRECISION=2 the f64 kernels only, 0 (default) both.  The
// Makefile builds the f64 TU without machine LICM: its pool kernel needs 143
// instead of 195 VGPRs that way, and same-box f64 frames ran 21-22 % faster
// (reflect_refract 1080p 1.337 -> 1.037 ms, cover 4K 4.91 -> 3.88 ms,
// three_sphere -6 %), while the f32 generic kernels were within -1..+3 %.
//
// Kind variants: built a second time with -DRTC_KINDS=<mask of shape kinds>
// -DRTC_VARIANT=<namespace>, the TU compiles the f32 pool kernel with the
// shape loops of those kinds only (rtc::<namespace>::launch_trace).  Same
// code for the kinds it keeps, so the same pixels; the host uses it for
// worlds whose kinds it covers (rtc_host.cpp, pool_variant).
#ifndef __HIPCC_RTC__  // hipRTC (per-scene build, rtc_jit.cpp) pre-includes the HIP runtime
#include <hip/hip_runtime.h>

#include <cstdint>
#endif

#include "rtc_internal.hpp"

namespace rtc {
#ifdef RTC_VARIANT
namespace RTC_VARIANT {
#endif

// ------------------------------------------------------------ real traits
template <typename R>
struct Real;

// RTC_F32_EXACT / RTC_F32_OFFSET / RTC_F32_REL_OFFSET: builds for the f32
// error study (tests/study_f32_error.py) — correctly rounded
// division, square root and pow instead of the hardware approximations, and
// other over/under-point offsets.  The product build uses none of them.
#ifndef RTC_F32_OFFSET
#define RTC_F32_OFFSET 1e-4f
#endif
#ifndef RTC_F32_REL_OFFSET
#define RTC_F32_REL_OFFSET 3e-5f
#endif
// Flat kinds (planes, cubes, triangles: t from one division per face, so
// the hit point is off the surface by a few ulps of the ray's coordinates):
// RTC_F32_FLAT_OFFSET x max(1, |p|inf, |o|inf) = 16 f32 ulps of the larger
// of hit point and ray origin.  RTC_F32_FLAT_KINDS: bit k = shape kind k
// takes it (0: every kind takes the quadric offset, round 5's product).
#ifndef RTC_F32_FLAT_OFFSET
#define RTC_F32_FLAT_OFFSET 1.9073486e-6f
#endif
#ifndef RTC_F32_FLAT_KINDS
#define RTC_F32_FLAT_KINDS 38
#endif
// Spheres: RTC_F32_SPHERE_OFFSET x max(1, |p|inf), 25 f32 ulps of |p|
// (cylinders and cones keep RTC_F32_REL_OFFSET: cylinders.yaml stands them
// on the floor, and smaller offsets meet the coplanar cap on the wrong side,
// DESIGN.md §4).  Round-6 study, 320x200 within 2/255 of the oracle at 3e-5
// -> 1e-5 -> 5e-6 -> 3e-6: refraction 0.97608 -> 0.98603 -> 0.98956 -> 0.99214,
// every other scene equal or closer.
#ifndef RTC_F32_SPHERE_OFFSET
#define RTC_F32_SPHERE_OFFSET 3e-6f
#endif
template <>
struct Real<float> {
    static constexpr float kEps = 8e-8f;        // guards (consts.rs:2)
    static constexpr float kOffset = RTC_F32_OFFSET;  // cap normals (8e-8 is below the
                                                      // f32 ulp at |y| > 0.7)
    static constexpr float kMax = __FLT_MAX__;  // consts.rs:8 analogue
    static constexpr float kInf = __builtin_huge_valf();
    // reference `a * b + c` (unfused there): fused here for throughput
    __device__ static inline float madd(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
    // reference `mul_add` sites
    __device__ static inline float rfma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
#ifdef RTC_F32_EXACT
    __device__ static inline float div(float a, float b) { return a / b; }
    __device__ static inline float sqrt(float a) { return __builtin_sqrtf(a); }
    __device__ static inline float rsqrt(float a) { return 1.0f / __builtin_sqrtf(a); }
    __device__ static inline float pow(float x, float y) { return __builtin_powf(x, y); }
#else
    __device__ static inline float div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
    __device__ static inline float sqrt(float a) { return __builtin_amdgcn_sqrtf(a); }
    __device__ static inline float rsqrt(float a) { return __builtin_amdgcn_rsqf(a); }
    __device__ static inline float pow(float x, float y) {  // x in (0, 1] here
        return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
    }
#endif
    __device__ static inline float floor(float a) { return __builtin_floorf(a); }
    __device__ static inline float trunc(float a) { return __builtin_truncf(a); }
    __device__ static inline float fabs(float a) { return __builtin_fabsf(a); }
    __device__ static inline float fmax(float a, float b) { return __builtin_fmaxf(a, b); }
    __device__ static inline float fmin(float a, float b) { return __builtin_fminf(a, b); }
    // over/under-point offset at hit point p (computed_hit.rs:33-34 uses
    // EPSILON = 8e-8, below the f32 ulp): RTC_F32_REL_OFFSET x max(1, |p|inf),
    // a fixed number of f32 ulps of p.  The error study: a fixed
    // 1e-4 put refraction.yaml 95.5 % within 2/255 of the oracle, a fixed
    // 1e-5 98.6 % but self-shadowed shadow_puppets' backdrop at |p| ~ 20
    // (97.2 %); the hardware rcp/sqrt/exp/log approximations change nothing.
    //
    // Round 6: planes and cubes take their own, smaller offset (above,
    // RTC_F32_FLAT_OFFSET): table.yaml floats its glass cube 1e-5 above the
    // table top (table.yaml:131-136), a tenth of 3e-5 x 3.45, so rays
    // reflected off the table under the cube started inside the glass and
    // table lost 3 % of its refractions.
    // cls: 0 sphere, 1 flat kind, 2 cylinder or cone (offset_class)
    __device__ static inline float surface_offset(float px, float py, float pz, float ox, float oy, float oz,
                                                  int cls) {
        const float mp = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(px), __builtin_fabsf(py)),
                                         __builtin_fmaxf(__builtin_fabsf(pz), 1.0f));
        const float mo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ox), __builtin_fabsf(oy)),
                                         __builtin_fmaxf(__builtin_fabsf(oz), mp));
        return cls == 1 ? RTC_F32_FLAT_OFFSET * mo : (cls == 0 ? RTC_F32_SPHERE_OFFSET : RTC_F32_REL_OFFSET) * mp;
    }
};

template <>
struct Real<double> {
    static constexpr double kEps = 0.00000008;
    static constexpr double kOffset = 0.00000008;  // computed_hit.rs:33-34
    static constexpr double kMax = __DBL_MAX__;
    static constexpr double kInf = __builtin_huge_val();
    __device__ static inline double madd(double a, double b, double c) { return a * b + c; }
    __device__ static inline double rfma(double a, double b, double c) { return __builtin_fma(a, b, c); }
    __device__ static inline double div(double a, double b) { return a / b; }
    __device__ static inline double sqrt(double a) { return __builtin_sqrt(a); }
    __device__ static inline double rsqrt(double a) { return 1.0 / __builtin_sqrt(a); }
    __device__ static inline double pow(double x, double y) { return ::pow(x, y); }
    __device__ static inline double floor(double a) { return __builtin_floor(a); }
    __device__ static inline double trunc(double a) { return __builtin_trunc(a); }
    __device__ static inline double fabs(double a) { return __builtin_fabs(a); }
    __device__ static inline double fmax(double a, double b) { return __builtin_fmax(a, b); }
    __device__ static inline double fmin(double a, double b) { return __builtin_fmin(a, b); }
    __device__ static inline double surface_offset(double, double, double, double, double, double, int) {
        return kOffset;
    }
};

template <typename R>
struct V3 {
    R x, y, z;
};

template <typename R>
__device__ inline V3<R> v3(R x, R y, R z) {
    return {x, y, z};
}
template <typename R>
__device__ inline V3<R> vsub(V3<R> a, V3<R> b) {
    return {a.x - b.x, a.y - b.y, a.z - b.z};
}
template <typename R>
__device__ inline V3<R> vneg(V3<R> a) {
    return {-a.x, -a.y, -a.z};
}
// vector.rs:93-95
template <typename R>
__device__ inline R dot(V3<R> a, V3<R> b) {
    return Real<R>::rfma(a.z, b.z, Real<R>::rfma(a.x, b.x, a.y * b.y));
}
// vector.rs:97-103
template <typename R>
__device__ inline V3<R> cross(V3<R> a, V3<R> b) {
    return {Real<R>::rfma(a.y, b.z, -a.z * b.y), Real<R>::rfma(a.z, b.x, -a.x * b.z),
            Real<R>::rfma(a.x, b.y, -a.y * b.x)};
}
// vector.rs:84-91
template <typename R>
__device__ inline V3<R> normalized(V3<R> v) {
    if constexpr (sizeof(R) == 4) {
        const R inv = Real<R>::rsqrt(Real<R>::madd(v.z, v.z, Real<R>::madd(v.y, v.y, v.x * v.x)));
        return {v.x * inv, v.y * inv, v.z * inv};
    } else {
        const R m = Real<R>::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
        return {v.x / m, v.y / m, v.z / m};
    }
}
template <typename R>
__device__ inline R magnitude(V3<R> v) {
    if constexpr (sizeof(R) == 4)
        return Real<R>::sqrt(Real<R>::madd(v.z, v.z, Real<R>::madd(v.y, v.y, v.x * v.x)));
    else
        return Real<R>::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
}
// vector.rs:105-107: v - (n * 2) * v.dot(n)
template <typename R>
__device__ inline V3<R> reflect(V3<R> v, V3<R> n) {
    const R d = dot(v, n);
    return {v.x - (n.x * R(2)) * d, v.y - (n.y * R(2)) * d, v.z - (n.z * R(2)) * d};
}
// ray.rs:30-32 / computed_hit.rs:33-34: p + d * t
template <typename R>
__device__ inline V3<R> along(V3<R> p, V3<R> d, R t) {
    return {Real<R>::madd(d.x, t, p.x), Real<R>::madd(d.y, t, p.y), Real<R>::madd(d.z, t, p.z)};
}

// Transform terms of the f32 path.  In a per-scene build (RTC_JIT) a shape
// record's matrix entries are compile-time constants, and most reference
// shapes are scaled and translated only: a 3x3 part with six exact zeros.
// A zero entry's term m * x is a signed zero, and adding a signed zero to a
// nonzero partial sum leaves it unchanged, so the term is dropped: 12 of the
// 21 transform operations of such a shape (the ray's components are finite on
// every lane whose result is used).  Only the sign of an exactly-zero
// coordinate can differ, and no later operation depends on it (divisions by
// a ray component are guarded by |d| >= EPSILON); the per-scene frames stay
// bit-identical to the generic kernel's (tests/test_gpu_jit.py).  The
// generic kernels read the records at run time and keep every term.
__device__ inline float kfma(float m, float x, float acc) {
#ifdef RTC_JIT
    if (__builtin_constant_p(m) && m == 0.0f) return acc;
#endif
    return __builtin_fmaf(m, x, acc);
}
__device__ inline float kmul(float m, float x) {
#ifdef RTC_JIT
    if (__builtin_constant_p(m) && m == 0.0f) return 0.0f;
#endif
    return m * x;
}

// matrix.rs:332-346 (w = 1), left fold from 0.0
template <typename R>
__device__ inline V3<R> xform_point(const R* m, V3<R> p) {
    if constexpr (sizeof(R) == 4) {
        return {kfma(m[2], p.z, kfma(m[1], p.y, kfma(m[0], p.x, m[3]))),
                kfma(m[6], p.z, kfma(m[5], p.y, kfma(m[4], p.x, m[7]))),
                kfma(m[10], p.z, kfma(m[9], p.y, kfma(m[8], p.x, m[11])))};
    } else {
        return {((((R)0 + m[0] * p.x) + m[1] * p.y) + m[2] * p.z) + m[3],
                ((((R)0 + m[4] * p.x) + m[5] * p.y) + m[6] * p.z) + m[7],
                ((((R)0 + m[8] * p.x) + m[9] * p.y) + m[10] * p.z) + m[11]};
    }
}
// matrix.rs:348-362 (w = 0)
template <typename R>
__device__ inline V3<R> xform_vector(const R* m, V3<R> v) {
    if constexpr (sizeof(R) == 4) {
        return {kfma(m[2], v.z, kfma(m[1], v.y, kmul(m[0], v.x))),
                kfma(m[6], v.z, kfma(m[5], v.y, kmul(m[4], v.x))),
                kfma(m[10], v.z, kfma(m[9], v.y, kmul(m[8], v.x)))};
    } else {
        return {(((R)0 + m[0] * v.x) + m[1] * v.y) + m[2] * v.z + m[3] * (R)0,
                (((R)0 + m[4] * v.x) + m[5] * v.y) + m[6] * v.z + m[7] * (R)0,
                (((R)0 + m[8] * v.x) + m[9] * v.y) + m[10] * v.z + m[11] * (R)0};
    }
}
// transpose(inverse) * n (shape.rs:25), 3x3 part
template <typename R>
__device__ inline V3<R> xform_normal(const R* m, V3<R> n) {
    if constexpr (sizeof(R) == 4) {
        return {kfma(m[8], n.z, kfma(m[4], n.y, kmul(m[0], n.x))),
                kfma(m[9], n.z, kfma(m[5], n.y, kmul(m[1], n.x))),
                kfma(m[10], n.z, kfma(m[6], n.y, kmul(m[2], n.x)))};
    } else {
        return {(((R)0 + m[0] * n.x) + m[4] * n.y) + m[8] * n.z,
                (((R)0 + m[1] * n.x) + m[5] * n.y) + m[9] * n.z,
                (((R)0 + m[2] * n.x) + m[6] * n.y) + m[10] * n.z};
    }
}

// f64/f32 `as i64` (saturating, NaN -> 0); only the parity bit is used
template <typename R>
__device__ inline bool odd_i64(R v) {
    if (!(v == v)) return false;                     // NaN -> 0
    const R lim = (R)9.2233720368547758e18;          // 2^63
    if (v >= lim) return true;                       // saturates to i64::MAX (odd)
    if (v <= -lim) return false;                     // saturates to i64::MIN (even)
    const long long i = (long long)v;
    return (i & 1) != 0;
}

// -------------------------------------------------------- shape intersect
// Each routine calls emit(t, valid) once per POTENTIAL entry, in the
// reference's push order; `valid` says whether the reference pushes it.
// Masks replace the reference's early returns so a wave never splits around
// a shape test: a divergent branch costs exec-mask SALU work and stalls
// (MI355X PMC: ~350 SALU per pixel-wave with branches), a select one VALU op.
// Masked-out lanes may compute inf/NaN; they are never emitted as valid.

// utils.rs:47-57; `ok` masks the caller's own guard
template <typename R, typename F>
__device__ inline void quadratic(R a, R b, R c, bool ok, F&& emit2) {
    const R disc = Real<R>::rfma((R)4 * a, -c, b * b);
    const bool v = ok && !(disc < (R)0);
    const R da = (R)2 * a;
    const R root = Real<R>::sqrt(disc);
    if constexpr (sizeof(R) == 4) {
        const R ri = __builtin_amdgcn_rcpf(da);
        emit2((-b - root) * ri, (-b + root) * ri, v);
    } else {
        emit2((-b - root) / da, (-b + root) / da, v);
    }
}

template <typename R>
__device__ inline R sel(bool c, R a, R b) {
    return c ? a : b;
}

// kNearest: the caller only wants the nearest t >= 0 of this shape (the
// closest-hit loop).  For a sphere or cube the two entries satisfy t1 <= t2
// with one validity, so t2 can only be that t when t1 < 0: emit one
// candidate instead of two (same result, half the hit bookkeeping).
template <typename R, int K, bool kNearest = false, typename F>
__device__ inline void entries(const ShapeRec<R>& s, V3<R> o, V3<R> d, F&& emit) {
    auto emit_pair = [&](R t1, R t2, bool v) {
        if constexpr (kNearest) {
            emit(sel(t1 >= (R)0, t1, t2), v);
        } else {
            emit(t1, v);
            emit(t2, v);
        }
    };
    using T = Real<R>;
    if constexpr (K == RT_SHAPE_SPHERE) {  // sphere.rs:41-53
        const R a = dot(d, d);
        const R b = (R)2 * dot(d, o);
        if constexpr (sizeof(R) == 4) {
            // b^2 - 4ac == 4 (a - |d x o|^2) (Lagrange's identity).  The
            // textbook form cancels catastrophically in f32 when the local
            // origin is far from the unit sphere (e.g. the backdrop of
            // shadow_puppets.yaml, a sphere scaled by 0.01 in z).
            const V3<R> c = cross(d, o);
            const R disc = (R)4 * (a - dot(c, c));
            const bool v = !(disc < (R)0);
            const R root = T::sqrt(disc);
            const R ri = __builtin_amdgcn_rcpf((R)2 * a);
            emit_pair((-b - root) * ri, (-b + root) * ri, v);
        } else {
            const R c = dot(o, o) - (R)1;
            quadratic<R>(a, b, c, true, emit_pair);
        }
    } else if constexpr (K == RT_SHAPE_PLANE) {  // plane.rs:42-48
        emit(T::div(-o.y, d.y), !(T::fabs(d.y) < T::kEps));
    } else if constexpr (K == RT_SHAPE_CUBE) {  // cube.rs:22-43, 65-85
        auto axis = [&](R org, R dir, R& lo, R& hi) {
            const R nmin = (R)-1 - org, nmax = (R)1 - org;
            const bool steep = T::fabs(dir) >= T::kEps;
            R l, h;
            if constexpr (sizeof(R) == 4) {
                const R r = sel(steep, __builtin_amdgcn_rcpf(dir), T::kMax);
                l = nmin * r;
                h = nmax * r;
            } else {
                l = sel(steep, nmin / dir, nmin * T::kMax);
                h = sel(steep, nmax / dir, nmax * T::kMax);
            }
            const bool swap = l > h;
            lo = sel(swap, h, l);
            hi = sel(swap, l, h);
        };
        R xn, xx, yn, yx, zn, zx;
        axis(o.x, d.x, xn, xx);
        axis(o.y, d.y, yn, yx);
        axis(o.z, d.z, zn, zx);
        const R tmin = T::fmax(T::fmax(T::fmax(-T::kMax, xn), yn), zn);
        const R tmax = T::fmin(T::fmin(T::fmin(T::kMax, xx), yx), zx);
        emit_pair(tmin, tmax, (tmin < tmax) & (tmax > (R)0));
    } else if constexpr (K == RT_SHAPE_CYLINDER || K == RT_SHAPE_CONE) {
        const R ymin = s.ymin, ymax = s.ymax;
        auto side = [&](R t1, R t2, bool v) {
            const bool swap = t1 > t2;
            const R lo = sel(swap, t2, t1), hi = sel(swap, t1, t2);
            R y1, y2;
            if constexpr (K == RT_SHAPE_CYLINDER) {  // cylinder.rs:96-104
                y1 = T::rfma(lo, d.y, o.y);
                y2 = T::rfma(hi, d.y, o.y);
            } else {  // cone.rs:99-107
                y1 = T::rfma(d.y, lo, o.y);
                y2 = T::rfma(d.y, hi, o.y);
            }
            emit(lo, v && ymin < y1 && y1 < ymax);
            emit(hi, v && ymin < y2 && y2 < ymax);
        };
        if constexpr (K == RT_SHAPE_CYLINDER) {  // cylinder.rs:81-110
            const R a = d.x * d.x + d.z * d.z;
            const R b = (R)2 * T::rfma(o.x, d.x, o.z * d.z);
            const R c = o.x * o.x + o.z * o.z - (R)1;
            quadratic<R>(a, b, c, T::fabs(a) > (R)0, side);
        } else {  // cone.rs:81-112
            const R a = d.x * d.x - d.y * d.y + d.z * d.z;
            const R b = (R)2 * T::rfma(o.z, d.z, T::rfma(o.x, d.x, -o.y * d.y));
            const R c = o.x * o.x - o.y * o.y + o.z * o.z;
            const bool single = T::fabs(a) < T::kEps && T::fabs(b) > T::kEps;
            emit(T::div(-c, (R)2 * b), single);
            quadratic<R>(a, b, c, !single, side);
        }
        // intersect_caps: cylinder.rs:41-58 / cone.rs:41-58
        const bool caps = (s.flags & kShapeClosed) && !(T::fabs(d.y) < T::kEps);
        const R r_lo = (K == RT_SHAPE_CYLINDER) ? (R)1 : ymin * ymin;
        const R r_hi = (K == RT_SHAPE_CYLINDER) ? (R)1 : ymax * ymax;
        R t = T::div(ymin - o.y, d.y);
        R x = T::rfma(d.x, t, o.x), z = T::rfma(d.z, t, o.z);
        emit(t, caps && x * x + z * z <= r_lo);
        t = T::div(ymax - o.y, d.y);
        x = T::rfma(d.x, t, o.x);
        z = T::rfma(d.z, t, o.z);
        emit(t, caps && x * x + z * z <= r_hi);
    } else {  // triangle.rs:39-56
        const V3<R> e1 = {s.tri[3], s.tri[4], s.tri[5]};
        const V3<R> e2 = {s.tri[6], s.tri[7], s.tri[8]};
        const V3<R> dce2 = cross(d, e2);
        const R det = dot(e1, dce2);
        const V3<R> v1o = vsub(o, V3<R>{s.tri[0], s.tri[1], s.tri[2]});
        const R u = T::div(dot(v1o, dce2), det);
        const V3<R> oce1 = cross(v1o, e1);
        const R v = T::div(dot(d, oce1), det);
        emit(T::div(dot(e2, oce1), det),
             !(T::fabs(det) < T::kEps) && (u >= (R)0 && u <= (R)1) && v > (R)0 && u + v < (R)1);
    }
}

// Copy a wave-uniform record.  The world tables reach the kernels as
// `const T* __restrict__` parameters (see scene_view): LLVM can then prove no
// store of the launch clobbers them and selects scalar s_load_dwordxN into
// SGPRs (free VALU operands) instead of per-lane global_loads.
template <typename T>
__device__ inline T ld_uniform(const T* p) {
    return *p;
}

#ifdef RTC_JIT
// Per-scene build (rtc_jit.cpp): the f32 shape table is a constexpr array
// (rtc_jit_scene.hpp, generated at upload) and each kind's loop is unrolled
// at compile time, so every record field is a constant of the instruction
// stream — no scalar loads, no loop control, no per-record branches.
template <int I, int E, typename F>
__device__ inline void jit_each(F&& f) {
    if constexpr (I < E) {
        f(jit::kShapes[I], I);
        jit_each<I + 1, E>(f);
    }
}
#endif

// Per-scene builds of worlds of at most 255 shapes take every value of the
// hit's shape record from the instruction stream: the hit's slot rides in
// the closest-hit key next to its world index, and its normal, material and
// pattern-space point come from one branch per slot present among the
// wave's hits, where the record is constants (jit_record_each).  Only the
// direct kernel is built so (rtc_jit.cpp make_request passes
// RTC_JIT_NO_RECORDS to pool builds, which measured faster with the records
// in LDS).
#if defined(RTC_JIT) && !defined(RTC_JIT_NO_RECORDS)
constexpr bool kJitRecords = jit::kBegin[kNumKinds] <= 255;  // rtc_host.cpp kJitRecordsMaxShapes
#else
constexpr bool kJitRecords = false;
#endif
#ifdef RTC_JIT
// The per-scene DIRECT kernel also takes the hit's material from constants
// and stages no LDS world at all (rtc_host.cpp plans it with none).
constexpr bool kJitConstMaterials = kJitRecords;
#endif

// Visit every shape of kind K (wave-uniform loop, scalar loads).
template <typename R, int K, typename F>
__device__ inline void for_kind(const DevScene<R>& sc, F&& f) {
#ifdef RTC_JIT
    if constexpr (sizeof(R) == 4) {
        jit_each<jit::kBegin[K], jit::kBegin[K + 1]>(f);
        return;
    }
#endif
    const int b = sc.kind_begin[K], e = sc.kind_begin[K + 1];
    for (int i = b; i < e; ++i) {
        const ShapeRec<R> s = ld_uniform(&sc.shapes[i]);
        f(s, i);
    }
}

#ifndef RTC_KINDS
#define RTC_KINDS 63  // every kind
#endif
template <typename R, int K, typename F>
__device__ inline void for_kind_if(const DevScene<R>& sc, F&& f) {
    if constexpr ((RTC_KINDS >> K) & 1) for_kind<R, K>(sc, f);
}

template <typename R, typename F>
__device__ inline void for_all_kinds(const DevScene<R>& sc, F&& f) {
    for_kind_if<R, RT_SHAPE_SPHERE>(sc, [&](const ShapeRec<R>& s, int i) { f.template operator()<RT_SHAPE_SPHERE>(s, i); });
    for_kind_if<R, RT_SHAPE_PLANE>(sc, [&](const ShapeRec<R>& s, int i) { f.template operator()<RT_SHAPE_PLANE>(s, i); });
    for_kind_if<R, RT_SHAPE_CUBE>(sc, [&](const ShapeRec<R>& s, int i) { f.template operator()<RT_SHAPE_CUBE>(s, i); });
    for_kind_if<R, RT_SHAPE_CYLINDER>(sc,
                                   [&](const ShapeRec<R>& s, int i) { f.template operator()<RT_SHAPE_CYLINDER>(s, i); });
    for_kind_if<R, RT_SHAPE_CONE>(sc, [&](const ShapeRec<R>& s, int i) { f.template operator()<RT_SHAPE_CONE>(s, i); });
    for_kind_if<R, RT_SHAPE_TRIANGLE>(sc,
                                   [&](const ShapeRec<R>& s, int i) { f.template operator()<RT_SHAPE_TRIANGLE>(s, i); });
}

// The roots of a kShapeSimilar sphere (f32), in world space: with oc = c - o
// and a = |d|^2, a t^2 - 2 t d.oc + |oc|^2 - r^2 = 0, whose discriminant is
// a r^2 - |d x oc|^2 (Lagrange's identity, as entries() forms it in object
// space), so t = (d.oc -+ sqrt(a r^2 - |d x oc|^2)) / a.  The same line and
// sphere as the object-space test (the transformation maps one onto the
// other), without transforming the ray: 3 subtractions instead of a point and
// a vector through the matrix, and 1/a once per ray (rdd) instead of a
// reciprocal per sphere.  f32 only: the f64 path keeps the reference's
// object-space arithmetic (its decisions must equal the oracle's).
template <typename R, bool kNearest, typename F>
__device__ inline void sphere_world(const ShapeRec<R>& s, V3<R> o, V3<R> d, R dd, R rdd, F&& emit) {
    const V3<R> oc = {s.tri[0] - o.x, s.tri[1] - o.y, s.tri[2] - o.z};
    const R tc = dot(d, oc);
    const V3<R> c = cross(d, oc);
    const R disc = s.tri[3] * dd - dot(c, c);
    const bool v = !(disc < (R)0);
    const R root = Real<R>::sqrt(disc);
    const R t1 = (tc - root) * rdd, t2 = (tc + root) * rdd;
    if constexpr (kNearest) {
        emit(sel(t1 >= (R)0, t1, t2), v);
    } else {
        emit(t1, v);
        emit(t2, v);
    }
}
// The slab test of a kShapeAxisAligned cube (f32), in world space.  With a
// diagonal linear part the object coordinate along axis i is s_i x_i + t_i,
// so entries()'s (-1 - lo_i) / ld_i is (w_i(-1) - o_i) / d_i, w_i(+-1) the
// world coordinates of the faces: one multiply by 1/d_i (rd, once per ray)
// per face instead of the ray's transform and three reciprocals per cube.  A
// parallel axis (|s_i d_i| < EPSILON, i.e. |d_i| below the record's
// threshold) takes sign(s_i) kMax as entries() takes kMax against the
// object-space numerator: the same signs, so the same slab decisions.  The
// swap, fmax/fmin order and validity are entries()'s.
template <typename R, bool kNearest, typename F>
__device__ inline void cube_world(const ShapeRec<R>& s, V3<R> o, V3<R> d, V3<R> rd, F&& emit) {
    using T = Real<R>;
    auto axis = [&](int i, R org, R dir, R rdir, R& lo, R& hi) {
        const bool steep = T::fabs(dir) >= s.tri[6 + i];
        const R r = sel(steep, rdir, s.tri[9 + i] * T::kMax);
        const R l = (s.tri[i] - org) * r, h = (s.tri[3 + i] - org) * r;
        const bool swap = l > h;
        lo = sel(swap, h, l);
        hi = sel(swap, l, h);
    };
    R xn, xx, yn, yx, zn, zx;
    axis(0, o.x, d.x, rd.x, xn, xx);
    axis(1, o.y, d.y, rd.y, yn, yx);
    axis(2, o.z, d.z, rd.z, zn, zx);
    const R tmin = T::fmax(T::fmax(T::fmax(-T::kMax, xn), yn), zn);
    const R tmax = T::fmin(T::fmin(T::fmin(T::kMax, xx), yx), zx);
    const bool v = (tmin < tmax) & (tmax > (R)0);
    if constexpr (kNearest) {
        emit(sel(tmin >= (R)0, tmin, tmax), v);
    } else {
        emit(tmin, v);
        emit(tmax, v);
    }
}
template <typename R, int K>
__device__ inline bool world_cube(const ShapeRec<R>& s) {
    if constexpr (sizeof(R) == 4 && K == RT_SHAPE_CUBE) return (s.flags & kShapeAxisAligned) != 0;
    return false;
}
template <typename R>
__device__ inline V3<R> recip3(V3<R> d) {
    if constexpr (sizeof(R) == 4)
        return {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z)};
    else return {(R)1 / d.x, (R)1 / d.y, (R)1 / d.z};
}
template <typename R, int K>
__device__ inline bool world_sphere(const ShapeRec<R>& s) {
    if constexpr (sizeof(R) == 4 && K == RT_SHAPE_SPHERE) return (s.flags & kShapeSimilar) != 0;
    return false;
}
template <typename R>
__device__ inline R recip(R x) {
    if constexpr (sizeof(R) == 4) return __builtin_amdgcn_rcpf(x);
    else return (R)1 / x;
}

// Wave-level cull (acceleration only): false when no active lane's ray
// o + t d, t >= 0, can meet the shape's padded world bounding sphere
// (rtc_host.cpp bounding_sphere), so the wave skips the shape; the reference
// tests every shape (world.rs:25-35) and the set of hits at t >= 0 is the
// same.  The ray meets the ball iff its line passes within r of the center,
// |d x oc|^2 <= r^2 |d|^2, and the center is not behind an outside origin
// (oc.d < 0 with |oc| > r makes |o + t d - C|^2 > r^2 for every t >= 0).
// The refractive-index walk counts t < 0 entries too and takes the line-only
// test below (wave_line_may_hit, per-scene builds).
// Wave-wide OR of a lane predicate (active lanes).  The raw builtin: HIP's
// __ballot(int) turns the predicate into a VGPR and compares it again.
__device__ inline bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// Per kind: planes are never bounded (no test, no record load); spheres and
// cubes always carry a radius, +inf when unbounded (RTC_DEBUG=cull=0 or a
// non-finite transform: every finite ray then passes), so their test has no
// branch on the record and its loads issue together; cylinders, cones and
// triangles keep a wave-uniform branch on r^2 < 0 (open cylinders and cones
// are unbounded, their test would be wasted VALU).
// dd = dot(d, d), formed once per ray by the caller: in the per-scene build
// the ray fence between unrolled shapes would otherwise recompute it for
// every shape.
// The ball test itself, for a shape's bound or (per-scene builds) a cluster
// of shapes' (for_all_culled): kHalfLine = t >= 0 only, else the whole line.
template <typename R, bool kHalfLine>
__device__ inline bool wave_ball_may_hit(R cx, R cy, R cz, R r2, V3<R> o, V3<R> d, R dd) {
    const V3<R> oc = {cx - o.x, cy - o.y, cz - o.z};
    // |d x oc|^2 = |oc|^2 |d|^2 - (oc.d)^2 (Lagrange): reuses oc.d of the
    // front test.  Rounding of the two products is bounded by ~12 ulp of
    // |oc|^2 |d|^2; shrinking |oc|^2 by 1 - kKeep (>> that) keeps the test
    // conservative, so no lane that meets the sphere is ever rejected.
    constexpr R kKeep = sizeof(R) == 4 ? (R)(1 - 1e-5) : (R)(1 - 1e-12);
    const R tc = dot(oc, d), oo = dot(oc, oc);
    if constexpr (!kHalfLine) return wave_any(Real<R>::madd(oo, kKeep, -r2) * dd <= tc * tc);
    // front = tc >= 0 | oo <= r2, lane = front & line test: one ballot per
    // comparison, combined as SGPR masks (a ballot of the combined bool makes
    // the compiler materialise it in a VGPR and compare it again: 2 VALU)
    const unsigned long long front = __builtin_amdgcn_ballot_w64(tc >= (R)0) | __builtin_amdgcn_ballot_w64(oo <= r2);
    return (front & __builtin_amdgcn_ballot_w64(Real<R>::madd(oo, kKeep, -r2) * dd <= tc * tc)) != 0;
}

template <typename R, int K>
__device__ inline bool wave_may_hit(const ShapeRec<R>& s, V3<R> o, V3<R> d, R dd) {
    if constexpr (K == RT_SHAPE_PLANE) return true;
    const R r2 = s.bound[3];  // radius^2
    if constexpr (K != RT_SHAPE_SPHERE && K != RT_SHAPE_CUBE)
        if (!(r2 >= (R)0)) return true;  // unbounded shape: wave-uniform
    return wave_ball_may_hit<R, true>(s.bound[0], s.bound[1], s.bound[2], r2, o, d, dd);
}

// The refractive-index walk's cull: entries at every t count there (t < 0
// included), so only the line test applies: no active lane's line passes
// within the bound's radius (|d x oc|^2 > r^2 |d|^2, with wave_may_hit's
// conservative margin) means no lane has an entry of this shape.  Per-scene
// builds only (constant bounds, kWalkCull); the generic kernel measured slower
// with it (round 2: its loads of the bound cost more than the scans it saved).
#ifndef RTC_WALK_CULL_MIN
#define RTC_WALK_CULL_MIN 4
#endif
template <typename R, int K>
__device__ inline bool wave_line_may_hit(const ShapeRec<R>& s, V3<R> o, V3<R> d, R dd) {
    if constexpr (K == RT_SHAPE_PLANE) return true;
    const R r2 = s.bound[3];
    if constexpr (K != RT_SHAPE_SPHERE && K != RT_SHAPE_CUBE)
        if (!(r2 >= (R)0)) return true;
    return wave_ball_may_hit<R, false>(s.bound[0], s.bound[1], s.bound[2], r2, o, d, dd);
}

// Per-scene build only: the ray's registers pass through an empty asm at the
// top of each unrolled shape, so the compiler cannot hoist every shape's
// ray-dependent terms (the cull's |o - c|^2, ...) to the front of the
// unrolled sequence, where they stay live and spill.  A no-op otherwise.
#ifndef RTC_JIT_FENCE_EVERY
#define RTC_JIT_FENCE_EVERY 1
#endif
// Worlds of fewer shapes than this take no fence at all (the direct kernel's
// builds: rtc_jit.cpp; the pool kernel's default 0 fences every world).
#ifndef RTC_JIT_FENCE_MIN_SHAPES
#define RTC_JIT_FENCE_MIN_SHAPES 0
#endif
template <typename R>
__device__ inline void jit_fence(V3<R>& o, V3<R>& d, int slot = 0) {
#if defined(RTC_JIT) && !defined(RTC_JIT_NO_FENCE)
    if constexpr (sizeof(R) == 4 && jit::kBegin[kNumKinds] >= RTC_JIT_FENCE_MIN_SHAPES)
        if (slot % RTC_JIT_FENCE_EVERY == 0)
            asm volatile("" : "+v"(o.x), "+v"(o.y), "+v"(o.z), "+v"(d.x), "+v"(d.y), "+v"(d.z));
#endif
}

// Every shape, as for_all_kinds, but per-scene builds of worlds with shape
// clusters (rtc_jit.cpp make_clusters) visit them cluster by cluster: a
// cluster's members only when some active lane's ray (kHalfLine) or line may
// meet the cluster's ball, which encloses every member's own padded ball, so
// a skipped member's own cull would have skipped it too.  Unclustered shapes
// (unbounded ones) are visited first.  The visit order differs from the table
// order; every caller's result is order-independent (closest hit by (t, world)
// key, any-hit by minimum, the walk per shape).
#ifdef RTC_JIT
constexpr int jit_kind_of(int slot) {
    int k = 0;
    while (k < kNumKinds - 1 && slot >= jit::kBegin[k + 1]) ++k;
    return k;
}
template <int M, typename F>
__device__ inline void jit_unclustered(F&& f) {
    if constexpr (M < jit::kNumUnclustered) {
        constexpr int slot = jit::kUnclustered[M];
        f.template operator()<jit_kind_of(slot)>(jit::kShapes[slot], slot);
        jit_unclustered<M + 1>(f);
    }
}
template <int C, int M, typename F>
__device__ inline void jit_members(F&& f) {
    if constexpr (M < jit::kClusterBegin[C + 1]) {
        constexpr int slot = jit::kClusterMembers[M];
        f.template operator()<jit_kind_of(slot)>(jit::kShapes[slot], slot);
        jit_members<C, M + 1>(f);
    }
}
// a cluster of spheres and cubes only (the walk's point test, refractive_indices)
template <int C>
constexpr bool jit_cluster_convex() {
    for (int m = jit::kClusterBegin[C]; m < jit::kClusterBegin[C + 1]; ++m) {
        const int k = jit_kind_of(jit::kClusterMembers[m]);
        if (k != RT_SHAPE_SPHERE && k != RT_SHAPE_CUBE) return false;
    }
    return true;
}
template <bool kHalfLine, int C, typename F, typename S>
__device__ inline void jit_clusters(V3<float>& o, V3<float>& d, float dd, F&& f, S&& skip) {
    if constexpr (C < jit::kNumClusters) {
        jit_fence(o, d);
        if (!skip(jit::kClusterBall[C][0], jit::kClusterBall[C][1], jit::kClusterBall[C][2], jit::kClusterBall[C][3],
                  jit_cluster_convex<C>()) &&
            wave_ball_may_hit<float, kHalfLine>(jit::kClusterBall[C][0], jit::kClusterBall[C][1], jit::kClusterBall[C][2],
                                                jit::kClusterBall[C][3], o, d, dd))
            jit_members<C, jit::kClusterBegin[C]>(f);
        jit_clusters<kHalfLine, C + 1>(o, d, dd, f, skip);
    }
}
#endif
// `skip(centre, r^2, convex)`: a caller's wave-uniform reason to pass a
// cluster by before its ball test (none by default); `convex`: every member
// is a sphere or a cube.
struct NoSkip {
    template <typename... A>
    __device__ bool operator()(A...) const {
        return false;
    }
};
template <typename R, bool kHalfLine, typename F, typename S = NoSkip>
__device__ inline void for_all_culled(const DevScene<R>& sc, V3<R>& o, V3<R>& d, R dd, F&& f, S&& skip = S{}) {
#ifdef RTC_JIT
    if constexpr (sizeof(R) == 4 && jit::kNumClusters > 0) {
        jit_unclustered<0>(f);
        jit_clusters<kHalfLine, 0>(o, d, dd, f, skip);
        return;
    }
#endif
    (void)o;
    (void)d;
    (void)dd;
    (void)skip;
    for_all_kinds<R>(sc, f);
}

template <typename R>
struct Hit {
    R t;
    int slot;   // index into the kind-sorted shape table, -1 = miss
    int world;  // world order, for the stable-sort tie rule
    int kind;
};

// Running first minimum of one ray over (t, world order), entries with
// t >= 0.  f32: (t, world) as one u64 key in a VGPR pair, compared once.
// tv + 0 maps -0 to +0, so every t >= 0 keys at or below +inf's bits while
// negative, invalid (-1) and NaN entries key above; the t kept is the
// entry's own.  The lane-mask form (f64, and f32 under RTC_VALU_KEYS=0)
// combines four compares bitwise (&& / || would be lowered to divergent
// branches), and those ANDs/ORs of wave masks are SALU instructions.
// Same-box A/B, keys vs masks (kernel time): three_sphere -2.8%,
// shadow_puppets -1.8%, reflect_refract -3.2%, table -1.4%, cover 0.
#ifndef RTC_VALU_KEYS
#define RTC_VALU_KEYS 1
#endif
template <typename R>
struct Nearest {
    static constexpr bool kKeys = sizeof(R) == 4 && RTC_VALU_KEYS;
    // per-scene records pack (world << 8 | slot) into the key's low word; only
    // the key form decodes it (hit() below)
    static_assert(!(kJitRecords && sizeof(R) == 4) || kKeys, "per-scene records need RTC_VALU_KEYS");
    R t = Real<R>::kInf;
    int w = __INT_MAX__;
    unsigned long long key = 0x7F8000007FFFFFFFull;  // (+inf, INT_MAX)
    __device__ inline void offer(R te, bool v, int we) {
        if constexpr (kKeys) {
            const float tv = v ? te : -1.0f;
            const unsigned long long k = ((unsigned long long)__float_as_uint(tv + 0.0f) << 32) | (uint32_t)we;
            const bool better = k < key;
            key = better ? k : key;
            t = better ? te : t;
        } else {
            const bool better = v & (te >= (R)0) & ((te < t) | ((te == t) & (we < w)));
            t = sel(better, te, t);
            w = better ? we : w;
        }
    }
    __device__ inline Hit<R> hit(const DevScene<R>& sc) const {
        const int hw = kKeys ? (int)(uint32_t)key : w;
        Hit<R> h{t, -1, hw, -1};
        if constexpr (kJitRecords && kKeys) {  // key = world << 8 | slot (closest_hit); kind unused
            if (hw != __INT_MAX__) {
                h.world = hw >> 8;
                h.slot = hw & 0xFF;
            }
            return h;
        }
        if (hw != __INT_MAX__) {
            const uint32_t ws = (uint32_t)sc.lworld_slot[hw];
            h.slot = (int)(ws & 0xFFFFFFu);
            h.kind = (int)(ws >> 24);
        }
        return h;
    }
};

// collect_intersections + hit (world.rs:25-35, intersections.rs:13-18):
// the first minimum t >= 0 in (t, world order, push order).  Within one
// shape a later entry never displaces an equal t (strict `w < world`), so
// push order needs no tracking; the loop carries (t, world) only and the
// slot/kind come from the world_slot table afterwards.
// Per-scene builds: does this cube hold one of the world's lights (1e-4 inside
// every face)?  Folded at compile time (constant record and lights): such a
// cube encloses the scene (table's room and walls), so most rays start inside.
#ifndef RTC_CUBE_EXIT_PATH
#define RTC_CUBE_EXIT_PATH 1
#endif
template <typename R>
__device__ inline bool jit_cube_holds_light(const ShapeRec<R>& s) {
#if defined(RTC_JIT) && RTC_CUBE_EXIT_PATH
    if constexpr (sizeof(R) == 4) {
        bool any = false;
        for (int i = 0; i < jit::kNumLights; ++i) {
            const V3<R> p = xform_point(s.inv, V3<R>{jit::kLights[i].position[0], jit::kLights[i].position[1],
                                                     jit::kLights[i].position[2]});
            constexpr R kIn = (R)(1 - 1e-4);
            any |= Real<R>::fabs(p.x) < kIn && Real<R>::fabs(p.y) < kIn && Real<R>::fabs(p.z) < kIn;
        }
        return any;
    }
#endif
    (void)s;
    return false;
}

// Acceleration-only skips on?  (RT_FLAG_NO_SKIPS turns them off to show they
// change nothing: a per-scene build compiles them out with RTC_NO_SKIPS, the
// generic kernels test the launch's flag, a wave-uniform SGPR.)
template <typename R>
__device__ inline bool skips_on(const DevScene<R>& sc) {
#ifdef RTC_NO_SKIPS
    (void)sc;
    return false;
#else
#ifdef RTC_JIT
    if constexpr (sizeof(R) == 4) return true;
#endif
    return !sc.no_skips;
#endif
}

template <typename R>
__device__ inline Hit<R> closest_hit(const DevScene<R>& sc, V3<R> o, V3<R> d) {
    Nearest<R> best;
    const R dd = dot(d, d), rdd = recip(dd);
    const V3<R> rd = recip3(d);
    for_all_culled<R, true>(sc, o, d, dd, [&]<int K>(const ShapeRec<R>& s, int slot) {
        jit_fence(o, d, slot);
        if (!wave_may_hit<R, K>(s, o, d, dd)) return;
        // (per-scene records: the slot rides below the world index; world
        // indices are distinct, so the order is the world order)
        const int w = kJitRecords && sizeof(R) == 4 ? (s.world_index << 8) | slot : s.world_index;
        if (world_sphere<R, K>(s)) {
            sphere_world<R, true>(s, o, d, dd, rdd, [&](R t, bool v) { best.offer(t, v, w); });
            return;
        }
        if (world_cube<R, K>(s)) {  // (an enclosing cube's exit too: tmin < 0 keeps tmax)
            cube_world<R, true>(s, o, d, rd, [&](R t, bool v) { best.offer(t, v, w); });
            return;
        }
        const V3<R> lo = xform_point(s.inv, o);
        const V3<R> ld = xform_vector(s.inv, d);
        if (K == RT_SHAPE_PLANE && skips_on(sc)) {
            // A plane's one entry is at t = -o_y / d_y (object space): with
            // o_y d_y > 0 (nonzero, one sign) it lies behind the origin and
            // cannot be the nearest t >= 0.  A wave whose every ray moves away
            // from the plane skips its division and bookkeeping: exact (the
            // product's sign is the signs' product; 0 and NaN never skip).
            if (!wave_any(!(lo.y * ld.y > (R)0))) return;
        }
        if constexpr (K == RT_SHAPE_CUBE && sizeof(R) == 4) {
            // A wave whose every origin lies strictly inside an enclosing cube:
            // each slab's entry is then negative and its exit positive, so the
            // nearest entry at t >= 0 is the exit, min over the slabs of the
            // larger bound, which is (+1 - o) r for r > 0 and (-1 - o) r for
            // r < 0: the same products and fmin order as entries(), without the
            // entry side.  (t > 0 keeps entries()'s validity bit for bit.)
            if (jit_cube_holds_light(s) && skips_on(sc) &&
                !wave_any(!(Real<R>::fabs(lo.x) < (R)1 && Real<R>::fabs(lo.y) < (R)1 && Real<R>::fabs(lo.z) < (R)1))) {
                using T = Real<R>;
                auto hi = [](auto org, auto dir) {  // (generic: never formed for f64)
                    const bool steep = T::fabs(dir) >= T::kEps;
                    const R r = sel(steep, __builtin_amdgcn_rcpf(dir), T::kMax);
                    return sel(r > (R)0, (R)1 - org, (R)-1 - org) * r;
                };
                const R tmax = T::fmin(T::fmin(T::fmin(T::kMax, hi(lo.x, ld.x)), hi(lo.y, ld.y)), hi(lo.z, ld.z));
                best.offer(tmax, tmax > (R)0, w);
                return;
            }
        }
        entries<R, K, true>(s, lo, ld, [&](R t, bool v) { best.offer(t, v, w); });
    });
    return best.hit(sc);
}

// is_in_shadow's test of one ray: some entry with 0 <= t < distance.  f32
// (RTC_VALU_KEYS): an unsigned min over the bits of (v ? t : -1) + 0 (the +0
// maps -0 to +0), so entries at t >= 0 order below +inf's bits and negative,
// invalid and NaN ones above; one compare with the distance at the end
// replaces three lane-mask AND/ORs per entry.
template <typename R>
struct Blocker {
    static constexpr bool kKeys = sizeof(R) == 4 && RTC_VALU_KEYS;
    bool hit = false;
    uint32_t tmin = 0x7F800000u;  // kKeys: bits of the nearest entry at t >= 0
    __device__ inline void offer(R t, bool v, R dist) {
        if constexpr (kKeys) {
            const uint32_t b = __float_as_uint((v ? t : -1.0f) + 0.0f);
            tmin = b < tmin ? b : tmin;
        } else {
            hit |= v & (t >= (R)0) & (t < dist);
        }
    }
    __device__ inline bool blocked(R dist) const {
        if constexpr (kKeys) return __uint_as_float(tmin) < dist;
        else return hit;
    }
};

// is_in_shadow (world.rs:98-112): any casting shape with 0 <= t < distance.
// lpos: the light the ray runs to (o + dist d).
template <typename R>
__device__ inline bool any_hit(const DevScene<R>& sc, V3<R> o, V3<R> d, R dist, V3<R> lpos) {
    Blocker<R> b;
    const R dd = dot(d, d), rdd = recip(dd);
    const V3<R> rd = recip3(d);
    // once every active lane is blocked the remaining clusters cannot change
    // the answer (per cluster, not per shape: a per-shape check measured
    // slower in round 3; per cluster cover -2.5 %, cylinders -4 %, table +1 %)
    const bool skips = skips_on(sc);
    auto skip = [&](R, R, R, R, bool) { return skips && !wave_any(!b.blocked(dist)); };
    for_all_culled<R, true>(sc, o, d, dd, [&]<int K>(const ShapeRec<R>& s, int slot) {
        if (!s.casts_shadow) return;  // wave-uniform
        jit_fence(o, d, slot);
        if (K == RT_SHAPE_CUBE && skips) {
            // A cube blocks the segment from o to the light only if no face
            // plane has both ends beyond it: one that does keeps the whole
            // segment outside (the cube is the intersection of its slabs).  A
            // wave whose every segment has such a face skips the cube (before
            // its cull: the light's object coordinates are constants in the
            // per-scene build).  Margins of 1e-5 relative keep the ends beyond
            // the face by far more than f32 rounding.  (Spheres, inside the same
            // box, measured slower: their cull is already tight.)
            const V3<R> po = xform_point(s.inv, o), pl = xform_point(s.inv, lpos);
            auto out = [](R a, R b) {
                const R lim_a = (R)1 + (R)1e-5 * ((R)1 + Real<R>::fabs(a));
                const R lim_b = (R)1 + (R)1e-5 * ((R)1 + Real<R>::fabs(b));
                return (a > lim_a && b > lim_b) || (a < -lim_a && b < -lim_b);
            };
            bool clear = out(po.x, pl.x) || out(po.y, pl.y) || out(po.z, pl.z);
            // Nor can a cube that holds the light (1e-4 inside every face) block
            // a segment starting strictly inside it: every slab's entry is then
            // at t < 0 and its exit beyond the light (table's room and walls,
            // each holding the points on the other).  Wave-uniform, and folded
            // at compile time in the per-scene build.
            constexpr R kIn = (R)(1 - 1e-4);
            if (Real<R>::fabs(pl.x) < kIn && Real<R>::fabs(pl.y) < kIn && Real<R>::fabs(pl.z) < kIn)
                clear = clear || (Real<R>::fabs(po.x) < (R)1 && Real<R>::fabs(po.y) < (R)1 && Real<R>::fabs(po.z) < (R)1);
            if (!wave_any(!clear)) return;
        }
        if (!wave_may_hit<R, K>(s, o, d, dd)) return;
        if (world_sphere<R, K>(s)) {
            sphere_world<R, false>(s, o, d, dd, rdd, [&](R t, bool v) { b.offer(t, v, dist); });
            return;
        }
        if (world_cube<R, K>(s)) {
            cube_world<R, false>(s, o, d, rd, [&](R t, bool v) { b.offer(t, v, dist); });
            return;
        }
        const V3<R> lo = xform_point(s.inv, o);
        if (K == RT_SHAPE_PLANE && skips) {
            // A plane blocks the segment from o to the light only if they lie on
            // opposite sides of it: with both on one side (object y of the same
            // sign) the crossing, if any, is behind o or beyond the light.  A wave
            // whose points all share the light's side skips the test.  The ratio
            // cap keeps the crossing beyond the light by far more than f32
            // rounding (|y_o| <= 1e4 |y_L|: beyond by a factor >= 1 + 1e-4).
            const R ly = xform_point(s.inv, lpos).y;
            if (!wave_any(!(lo.y * ly > (R)0 && Real<R>::fabs(lo.y) <= (R)1e4 * Real<R>::fabs(ly)))) return;
        }
        const V3<R> ld = xform_vector(s.inv, d);
        entries<R, K>(s, lo, ld, [&](R t, bool v) { b.offer(t, v, dist); });
    }, skip);
    return b.blocked(dist);
}

// Refractive-index containers walk (intersection.rs:33-62) without a list.
// The list holds at most one member of each identity class (value-equal
// shapes, rtc_internal.hpp kShapeClassEnd): an entry of a shape removes the
// class's member if one is present (position() compares by value,
// intersection.rs:47) and pushes the shape otherwise.  So a class is in the
// list at the hit iff an odd number of its members' entries sort before the
// hit, and the list's `last()` is the present class whose latest such entry
// sorts latest.  Keys sort by (t, world order, push order).  Members of a
// class are adjacent in the table, so the count and latest key run over a
// class's records and are settled at its last one.  kDup = false (a world
// with no value-equal shapes, the common case) compiles the walk with one
// class per record: every record ends its class and the class is the slot.
// Same-box A/B, per-class walk in every world vs this split: reflect_refract
// +3.5%, refraction +2.2% kernel time.
template <typename R, bool kDup>
__device__ inline void refractive_indices(const DevScene<R>& sc, V3<R> o, V3<R> d, const Hit<R>& h, int hit_mat,
                                          R& n1, R& n2) {
    struct Key {
        R t;
        int w, e;
    };
    auto before = [](const Key& a, const Key& b) {
        return a.t < b.t || (a.t == b.t && (a.w < b.w || (a.w == b.w && a.e < b.e)));
    };
    // The hit's own entry is the first of its shape at t == h.t, so entries
    // of that shape sort before it iff t < h.t: push order 0 says exactly that.
    const Key hk{h.t, h.world, 0};
    // The three flags share one word: as separate bools, the compiler merged
    // the branches' stores into one store through a selected pointer, which
    // put the flags in scratch (a scratch store and load per shape).
    constexpr int kHaveAll = 1, kHaveOther = 2, kHitPresent = 4;
    int flags = 0;
    Key best_all{}, best_other{};
    int mat_all = -1, mat_other = -1;
    // a class whose entries before the hit are odd in number is in the list
    auto settle = [&](int count, const Key& last, const ShapeRec<R>& s, bool is_hit_class) {
        if (count & 1) {
            if (!(flags & kHaveAll) || before(best_all, last)) {
                best_all = last;
                mat_all = s.material;
                flags |= kHaveAll;
            }
            if (is_hit_class) {
                flags |= kHitPresent;
            } else if (!(flags & kHaveOther) || before(best_other, last)) {
                best_other = last;
                mat_other = s.material;
                flags |= kHaveOther;
            }
        }
    };
    // entries of one shape before the hit: their count and the latest
    auto scan = [&]<int K>(const ShapeRec<R>& s, int& count, Key& last) {
        jit_fence(o, d);
        const int w = s.world_index;
        int e = 0;
        auto take = [&](R t, bool v) {
            const Key k{t, w, e};
            if (v && before(k, hk)) {
                ++count;
                if (count == 1 || before(last, k)) last = k;
            }
            e += v ? 1 : 0;
        };
        if (world_sphere<R, K>(s)) {  // (the same roots as closest_hit's)
            const R dd = dot(d, d);
            sphere_world<R, false>(s, o, d, dd, recip(dd), take);
            return;
        }
        if (world_cube<R, K>(s)) {  // (the same slabs as closest_hit's)
            cube_world<R, false>(s, o, d, recip3(d), take);
            return;
        }
        entries<R, K>(s, xform_point(s.inv, o), xform_vector(s.inv, d), take);
    };
#if defined(RTC_JIT) && !defined(RTC_NO_WALK_CULL)
    // worlds of a few bounded shapes (refraction.yaml: a lens of two spheres
    // over a plane) have nothing to cull: every line meets the lens's bounds,
    // and the tests cost 2.4 % there; from RTC_WALK_CULL_MIN bounded shapes on
    // they pay (cover 1080p -16 %, reflect_refract -2 %)
    constexpr int kBounded = jit::kBegin[kNumKinds] - (jit::kBegin[RT_SHAPE_PLANE + 1] - jit::kBegin[RT_SHAPE_PLANE]);
    constexpr bool kWalkCull = sizeof(R) == 4 && kBounded >= RTC_WALK_CULL_MIN;
#else
    constexpr bool kWalkCull = false;
#endif
    const R dd = dot(d, d);
    if constexpr (kDup) {
        const uint32_t hit_class = (uint32_t)sc.lshapes[h.slot].flags >> kShapeClassShift;
        int count = 0;  // over the current class's records
        Key last{};
        for_all_kinds<R>(sc, [&]<int K>(const ShapeRec<R>& s, int slot) {
            if (!kWalkCull || wave_line_may_hit<R, K>(s, o, d, dd)) scan.template operator()<K>(s, count, last);
            if (!(s.flags & kShapeClassEnd)) return;  // wave-uniform: more members follow
            settle(count, last, s, (uint32_t)s.flags >> kShapeClassShift == hit_class);
            count = 0;
        });
    } else if constexpr (kWalkCull) {  // (line culls: clusters too in per-scene builds)
        // Only a shape with an odd count of entries before the hit is settled.
        // A sphere's or cube's two entries t1 <= t2 share one validity, so its
        // count is odd only when t1 sorts before the hit and t2 does not: the
        // hit point p = o + t d lies between them, inside the shape.  A sphere
        // or cube (or a cluster of them) whose padded ball holds no active
        // lane's p, and which is no lane's hit shape, settles nothing and is
        // skipped: a test of p against the ball in place of the line test,
        // and far stronger (the line passes near many shapes its hit point is
        // nowhere near).  Conservative like the line test: the pad
        // (rtc_host.cpp bounding_sphere, >= 1e-4 of the ball's distance from
        // the origin) dwarfs p's rounding, and |p - c|^2 is shrunk by kKeep.
        // Other kinds keep the line test: an open cylinder's or cone's walls,
        // and a triangle, leave odd counts far from the shape (one entry
        // before the hit, the other missing).  Frames equal the line-culled
        // walk's bit for bit (tests/test_gpu_skips.py renders against
        // RT_FLAG_NO_SKIPS, which keeps the line test).
        const bool points = skips_on(sc);
        // (p - c formed per test from o, d and t, which stay live for the
        // scans anyway: a p held across the walk spilled in cover's build)
        auto holds = [&](R cx, R cy, R cz, R r2) {
            constexpr R kKeep = sizeof(R) == 4 ? (R)(1 - 1e-5) : (R)(1 - 1e-12);
            const V3<R> pc = {Real<R>::madd(h.t, d.x, o.x - cx), Real<R>::madd(h.t, d.y, o.y - cy),
                              Real<R>::madd(h.t, d.z, o.z - cz)};
            return wave_any(dot(pc, pc) * kKeep <= r2);
        };
        for_all_culled<R, false>(sc, o, d, dd, [&]<int K>(const ShapeRec<R>& s, int slot) {
            if (points && (K == RT_SHAPE_SPHERE || K == RT_SHAPE_CUBE)) {
                if (!holds(s.bound[0], s.bound[1], s.bound[2], s.bound[3]) && !wave_any(slot == h.slot)) return;
            } else if (!wave_line_may_hit<R, K>(s, o, d, dd)) {
                return;  // no entries: nothing to settle
            }
            int count = 0;
            Key last{};
            scan.template operator()<K>(s, count, last);
            settle(count, last, s, slot == h.slot);
        }, [&](R cx, R cy, R cz, R r2, bool convex) {
            // a cluster of spheres and cubes whose ball holds no lane's p (a
            // hit shape's own ball holds its p, so the hit's cluster stays)
            return points && convex && !holds(cx, cy, cz, r2);
        });
    } else {
        for_all_kinds<R>(sc, [&]<int K>(const ShapeRec<R>& s, int slot) {
            int count = 0;
            Key last{};
            scan.template operator()<K>(s, count, last);
            settle(count, last, s, slot == h.slot);
        });
    }
    n1 = (flags & kHaveAll) ? sc.lmats[mat_all].refractive_index : (R)1;
    if (flags & kHitPresent)  // the hit's class leaves the list
        n2 = (flags & kHaveOther) ? sc.lmats[mat_other].refractive_index : (R)1;
    else              // the hit pushes itself
        n2 = sc.lmats[hit_mat].refractive_index;
}

// local_normal_at of each shape (object space, not normalized)
template <typename R>
__device__ inline V3<R> local_normal(const ShapeRec<R>& s, int kind, V3<R> lp) {
    using T = Real<R>;
    V3<R> ln;
    switch (kind) {
        case RT_SHAPE_SPHERE: ln = lp; break;                          // sphere.rs:57-59
        case RT_SHAPE_PLANE: ln = {(R)0, (R)1, (R)0}; break;          // plane.rs:52-54
        case RT_SHAPE_CUBE: {                                          // cube.rs:89-101
            const R ax = T::fabs(lp.x), ay = T::fabs(lp.y), az = T::fabs(lp.z);
            const R mx = T::fmax(T::fmax(T::fmax(-T::kMax, ax), ay), az);
            auto near = [](R a, R b) { return a == b || T::fabs(a - b) < T::kEps; };
            if (near(mx, ax)) ln = {lp.x, (R)0, (R)0};
            else if (near(mx, ay)) ln = {(R)0, lp.y, (R)0};
            else ln = {(R)0, (R)0, lp.z};
            break;
        }
        case RT_SHAPE_CYLINDER: {  // cylinder.rs:114-126
            const R dist = lp.x * lp.x + lp.z * lp.z;
            if (dist < (R)1 && lp.y >= s.ymax - T::kOffset) ln = {(R)0, (R)1, (R)0};
            else if (dist < (R)1 && lp.y <= s.ymin + T::kOffset) ln = {(R)0, (R)-1, (R)0};
            else ln = {lp.x, (R)0, lp.z};
            break;
        }
        case RT_SHAPE_CONE: {  // cone.rs:116-133
            const R dist = lp.x * lp.x + lp.z * lp.z;
            if (dist < s.ymax * s.ymax && lp.y >= s.ymax - T::kOffset) ln = {(R)0, (R)1, (R)0};
            else if (dist < s.ymin * s.ymin && lp.y <= s.ymin + T::kOffset) ln = {(R)0, (R)-1, (R)0};
            else {
                R y = T::sqrt(dist);
                if (lp.y > (R)0) y = -y;
                ln = {lp.x, y, lp.z};
            }
            break;
        }
        default: ln = {s.tri[9], s.tri[10], s.tri[11]}; break;  // triangle.rs:78-80
    }
    return ln;
}

// shape.rs:22-27: world point -> object point -> local normal -> world normal
template <typename R>
__device__ inline V3<R> normal_at(const ShapeRec<R>& s, int kind, V3<R> p) {
    return normalized(xform_normal(s.inv, local_normal(s, kind, xform_point(s.inv, p))));
}

#ifdef RTC_JIT
// Per-scene build of a small world: the hit's normal from the constant
// record of its slot.  Each slot present among a wave's hits runs its own
// case (an exec-masked branch per slot), where the kind is known and the
// record's matrix is made of immediates: a plane's world normal before
// normalisation is a constant, a scaled sphere's transforms lose their zero
// terms (kfma).  The generic path reads the record from LDS and runs every
// kind's transforms.  The unnormalised normal passes an empty asm so the
// hardware rsq runs as in the generic kernel (the compiler would fold it for
// a constant with a correctly rounded 1/sqrt): frames stay bit-identical.
#ifndef RTC_JIT_NORMAL_MAX
#define RTC_JIT_NORMAL_MAX 8
#endif
template <int I>
constexpr int jit_kind_of() {
    int k = 0;
    while (jit::kBegin[k + 1] <= I) ++k;
    return k;
}
template <int I, int E>
__device__ inline void jit_normal_each(int slot, V3<float> p, V3<float>& w) {
    if constexpr (I < E) {
        if (slot == I) {
            const ShapeRec<float>& s = jit::kShapes[I];
            w = xform_normal(s.inv, local_normal(s, jit_kind_of<I>(), xform_point(s.inv, p)));
        }
        jit_normal_each<I + 1, E>(slot, p, w);
    }
}

// kJitRecords: the hit's unnormalised world normal and material index, and
// (jit_object_each) the object-space point of p, from a branch per slot
template <int I, int E>
__device__ inline void jit_record_each(int slot, V3<float> p, V3<float>& w, int& mat) {
    if constexpr (I < E) {
        if (slot == I) {
            const ShapeRec<float>& s = jit::kShapes[I];
            w = xform_normal(s.inv, local_normal(s, jit_kind_of<I>(), xform_point(s.inv, p)));
            mat = s.material;
        }
        jit_record_each<I + 1, E>(slot, p, w, mat);
    }
}
// ... and, for the direct kernel, the hit's material as constants too
// (jit::kMaterials: registers instead of an LDS world and its staging)
template <int I, int E>
__device__ inline void jit_record_material_each(int slot, V3<float> p, V3<float>& w, MaterialRec<float>& mat) {
    if constexpr (I < E) {
        if (slot == I) {
            const ShapeRec<float>& s = jit::kShapes[I];
            w = xform_normal(s.inv, local_normal(s, jit_kind_of<I>(), xform_point(s.inv, p)));
            mat = jit::kMaterials[s.material];
        }
        jit_record_material_each<I + 1, E>(slot, p, w, mat);
    }
}
template <int I, int E>
__device__ inline void jit_object_each(int slot, V3<float> p, V3<float>& obj) {
    if constexpr (I < E) {
        if (slot == I) obj = xform_point(jit::kShapes[I].inv, p);
        jit_object_each<I + 1, E>(slot, p, obj);
    }
}
#endif

template <typename R>
__device__ inline V3<R> hit_normal(const ShapeRec<R>& s, int slot, int kind, V3<R> p) {
#ifdef RTC_JIT
    if constexpr (sizeof(R) == 4 && jit::kBegin[kNumKinds] <= RTC_JIT_NORMAL_MAX) {
        V3<float> w = {0.0f, 0.0f, 0.0f};
        jit_normal_each<0, jit::kBegin[kNumKinds]>(slot, p, w);
        asm volatile("" : "+v"(w.x), "+v"(w.y), "+v"(w.z));
        return normalized(w);
    }
#endif
    (void)slot;
    return normal_at(s, kind, p);
}

// Pattern::color_at_shape (pattern.rs:10-14) and the five color_at bodies.
// A per-scene build compiles in only the kinds its world's table holds
// (jit::kPatternKinds: the walk can meet no other).
#ifdef RTC_JIT
#define RTC_PATTERN_KIND(k) \
    if (!((jit::kPatternKinds >> (k)) & 1u)) __builtin_unreachable()
#else
#define RTC_PATTERN_KIND(k) (void)0
#endif
template <typename R>
__device__ inline V3<R> pattern_color_obj(const DevScene<R>& sc, int pid, V3<R> obj) {  // obj: object space
    using T = Real<R>;
    const PatternRec<R>* pr = &sc.lpats[pid];
    const V3<R> pp = xform_point(pr->inv, obj);
    for (int guard = 0; guard < 16; ++guard) {
        switch (pr->kind) {
            case RT_PATTERN_STRIPE:  // stripe_pattern.rs:24-31
                RTC_PATTERN_KIND(RT_PATTERN_STRIPE);
                return odd_i64(T::floor(pp.x)) ? v3(pr->color_b[0], pr->color_b[1], pr->color_b[2])
                                                : v3(pr->color_a[0], pr->color_a[1], pr->color_a[2]);
            case RT_PATTERN_GRADIENT: {  // gradient_pattern.rs:24-31 (ping-pong)
                RTC_PATTERN_KIND(RT_PATTERN_GRADIENT);
                R f = T::fabs(pp.x - T::trunc(pp.x));
                if (odd_i64(pp.x)) f = (R)1 - f;
                return {pr->color_a[0] + (pr->color_b[0] - pr->color_a[0]) * f,
                        pr->color_a[1] + (pr->color_b[1] - pr->color_a[1]) * f,
                        pr->color_a[2] + (pr->color_b[2] - pr->color_a[2]) * f};
            }
            case RT_PATTERN_RING: {  // ring_pattern.rs:25-32
                RTC_PATTERN_KIND(RT_PATTERN_RING);
                const R r = T::floor(T::sqrt(pp.x * pp.x + pp.z * pp.z));
                return odd_i64(r) ? v3(pr->color_b[0], pr->color_b[1], pr->color_b[2])
                                  : v3(pr->color_a[0], pr->color_a[1], pr->color_a[2]);
            }
            case RT_PATTERN_CHECKER: {  // checker_pattern.rs:24-31
                RTC_PATTERN_KIND(RT_PATTERN_CHECKER);
                const R sum = T::floor(pp.x) + T::floor(pp.y) + T::floor(pp.z);
                return odd_i64(sum) ? v3(pr->color_b[0], pr->color_b[1], pr->color_b[2])
                                    : v3(pr->color_a[0], pr->color_a[1], pr->color_a[2]);
            }
            case RT_PATTERN_COMPLEX:  // complex_pattern.rs:25-32: sub transforms ignored
                RTC_PATTERN_KIND(RT_PATTERN_COMPLEX);
                pr = &sc.lpats[odd_i64(T::floor(pp.x)) ? pr->sub_b : pr->sub_a];
                continue;
            default:  // TestPattern (pattern.rs:55-58)
                RTC_PATTERN_KIND(RT_PATTERN_TEST);
                return pp;
        }
    }
    return {(R)0, (R)0, (R)0};
}
template <typename R>
__device__ inline V3<R> pattern_color(const DevScene<R>& sc, int pid, const ShapeRec<R>& s, V3<R> p) {
    return pattern_color_obj(sc, pid, xform_point(s.inv, p));
}

// Per-thread event counters (rt_stats order).
// Event counters of one wave (rt_stats order), kept wave-uniform: each
// event is counted as popcount(ballot(flag)) at a point every lane of the
// wave reaches, so the counters live in SGPRs (per-lane counters cost 8
// VGPRs, a v_add per event and a 48-shuffle reduction per wave).
struct Counts {
    uint32_t c[kNumCounters];
};

__device__ inline uint32_t wave_count(bool p) {
    return (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(p));
}

// One radiance ray: closest hit, shading over all lights with shadow rays,
// and the (at most two) children.  Returns false on a miss.
template <typename R>
struct Shaded {
    V3<R> surface;  // Σ_lights lighting(...)  (world.rs:44-52)
    bool refl_child = false, refr_child = false;
    bool patterned = false;  // each light evaluation samples a pattern
    bool refr_eval = false;  // refracted_color past the opaque/depth check
    bool schlick = false;    // schlicks_approximation evaluated
};

// Children are handed to push(origin, direction, weight) where they are
// made (weight: reflectiveness × {R | 1}, transparency × {1-R | 1}), not
// returned: holding both children until the caller's pushes kept ~14 more
// values live through the refraction code and forced spills.
struct NoPush {
    template <typename V, typename R>
    __device__ void operator()(V, V, R) const {}
};

// RT_FLAG_GENERATIONS (generic kernels only; a diagnostic frame, e.g. the
// bench's per-generation line): the wave's traced rays and shaded hits by
// `remaining`, one pass per distinct value among the traced lanes and one
// global atomic pair per pass from lane 0.  Call where every lane arrives.
__device__ inline void count_generations(unsigned long long* gc, bool traced, bool shaded, uint32_t rem) {
    unsigned long long left = __builtin_amdgcn_ballot_w64(traced);
    while (left) {
        const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)rem, (int)__builtin_ctzll(left));
        const unsigned long long same = __builtin_amdgcn_ballot_w64(traced && rem == r);
        const unsigned long long hit = __builtin_amdgcn_ballot_w64(shaded && rem == r);
        if ((threadIdx.x & 63) == 0 && r < (uint32_t)kGenSlots) {
            atomicAdd(&gc[r], (unsigned long long)__builtin_popcountll(same));
            if (hit) atomicAdd(&gc[kGenSlots + r], (unsigned long long)__builtin_popcountll(hit));
        }
        left &= ~same;
    }
}

// Count one wave's events after shading (call where every lane arrives):
// `primary` rays entering the path, `hit` = shade_ray's result.
template <typename R>
__device__ inline void count_events(Counts& k, bool primary, bool hit, const Shaded<R>& sh, int n_lights) {
    k.c[0] += wave_count(primary);
    const uint32_t shaded = wave_count(hit);
    k.c[4] += shaded;
    k.c[1] += shaded * (uint32_t)n_lights;  // world.rs:46-52: one shadow ray per light
    k.c[5] += wave_count(hit & sh.patterned) * (uint32_t)n_lights;
    k.c[2] += wave_count(hit & sh.refl_child);
    k.c[3] += wave_count(hit & sh.refr_child);
    k.c[6] += wave_count(hit & sh.refr_eval);
    k.c[7] += wave_count(hit & sh.schlick);
}

// prepare_computations (intersection.rs:21-31) up to the colour the lights
// see: the hit point, the normal turned toward the eye, over_point
// (computed_hit.rs:33) and the surface colour there (material.rs:75-80: a
// pattern is sampled at over_point, once per hit).  Returns the material.
template <typename R>
struct Prepared {
    V3<R> p, n, eye, over, base;
    R off;    // the over/under-point offset (computed_hit.rs:33-34; f32: per kind)
    int mat;  // the hit's material index
};

// The hit's offset class for Real<float>::surface_offset: 1 for the flat
// kinds of RTC_F32_FLAT_KINDS, 0 for spheres, 2 otherwise.  Per-scene builds
// with records know the kind from the slot's range (constants).
__device__ inline int offset_class_of_kind(int kind) {
    return ((RTC_F32_FLAT_KINDS >> (kind & 31)) & 1) ? 1 : (kind == RT_SHAPE_SPHERE ? 0 : 2);
}

template <typename R>
__device__ inline int offset_class(const Hit<R>& h) {
#ifdef RTC_JIT
    if constexpr (sizeof(R) == 4) {
        int c = 2;
#pragma unroll
        for (int k = 0; k < kNumKinds; ++k)
            if (h.slot >= jit::kBegin[k] && h.slot < jit::kBegin[k + 1]) c = offset_class_of_kind(k);
        return c;
    }
#endif
    return offset_class_of_kind(h.kind);
}

template <typename R>
__device__ inline R hit_offset(const Hit<R>& h, V3<R> p, V3<R> o) {
    return Real<R>::surface_offset(p.x, p.y, p.z, o.x, o.y, o.z, offset_class(h));
}

#ifdef RTC_JIT
// The per-scene direct kernel (no pool, few live values): prepare_hit with
// the material as constants of the slot's branch (kJitConstMaterials).
__device__ inline void prepare_hit_const(const DevScene<float>& sc, V3<float> o, V3<float> d, const Hit<float>& h,
                                         Prepared<float>& q, bool& patterned, MaterialRec<float>& m) {
    q.p = along(o, d, h.t);
    V3<float> w = {0.0f, 0.0f, 0.0f};
    jit_record_material_each<0, jit::kBegin[kNumKinds]>(h.slot, q.p, w, m);
    asm volatile("" : "+v"(w.x), "+v"(w.y), "+v"(w.z));  // the hardware rsq, as hit_normal (bit for bit)
    q.n = normalized(w);
    q.eye = vneg(d);
    if (dot(q.n, q.eye) < 0.0f) q.n = vneg(q.n);
    q.mat = -1;  // (the direct kernel walks no refractive indices)
    q.off = hit_offset(h, q.p, o);
    q.over = along(q.p, q.n, q.off);
    q.base = {m.color[0], m.color[1], m.color[2]};
    patterned = m.pattern >= 0;
    if (jit::kPatterns && patterned) {
        V3<float> obj = {0.0f, 0.0f, 0.0f};
        jit_object_each<0, jit::kBegin[kNumKinds]>(h.slot, q.over, obj);
        q.base = pattern_color_obj(sc, m.pattern, obj);
    }
}
#endif

template <typename R>
__device__ inline const MaterialRec<R>& prepare_hit(const DevScene<R>& sc, V3<R> o, V3<R> d, const Hit<R>& h,
                                                     Prepared<R>& q, bool& patterned) {
#ifdef RTC_JIT
    if constexpr (kJitRecords && sizeof(R) == 4) {
        q.p = along(o, d, h.t);
        V3<float> w = {0.0f, 0.0f, 0.0f};
        int mat = 0;
        jit_record_each<0, jit::kBegin[kNumKinds]>(h.slot, q.p, w, mat);
        asm volatile("" : "+v"(w.x), "+v"(w.y), "+v"(w.z));  // the hardware rsq, as hit_normal (bit for bit)
        q.n = normalized(w);
        q.eye = vneg(d);
        if (dot(q.n, q.eye) < (R)0) q.n = vneg(q.n);
        q.mat = mat;
        const MaterialRec<R>& m = sc.lmats[mat];
        q.off = hit_offset(h, q.p, o);
        q.over = along(q.p, q.n, q.off);
        q.base = {m.color[0], m.color[1], m.color[2]};
        patterned = m.pattern >= 0;
        if (jit::kPatterns && patterned) {
            V3<float> obj = {0.0f, 0.0f, 0.0f};
            jit_object_each<0, jit::kBegin[kNumKinds]>(h.slot, q.over, obj);
            q.base = pattern_color_obj(sc, m.pattern, obj);
        }
        return m;
    }
#endif
    const ShapeRec<R>& s = sc.lshapes[h.slot];
    q.p = along(o, d, h.t);
    q.n = hit_normal(s, h.slot, h.kind, q.p);
    q.eye = vneg(d);
    if (dot(q.n, q.eye) < (R)0) q.n = vneg(q.n);
    q.mat = s.material;
    const MaterialRec<R>& m = sc.lmats[s.material];
    q.off = hit_offset(h, q.p, o);
        q.over = along(q.p, q.n, q.off);
    q.base = {m.color[0], m.color[1], m.color[2]};
    patterned = m.pattern >= 0;
#ifdef RTC_JIT
    constexpr bool kPatterns = jit::kPatterns;  // per-scene build: no pattern in the world, no pattern code
#else
    constexpr bool kPatterns = true;
#endif
    if (kPatterns && patterned) q.base = pattern_color(sc, m.pattern, s, q.over);
    return m;
}

// The world's lights in order: per-scene builds unroll them with their
// records as constants (rtc_jit.cpp scene_header); the generic kernels read
// them wave-uniformly.
#ifdef RTC_JIT
template <int I, int E, typename F>
__device__ inline void jit_light_each(F&& f) {
    if constexpr (I < E) {
        f(jit::kLights[I]);
        jit_light_each<I + 1, E>(f);
    }
}
#endif
template <typename R, typename F>
__device__ inline void for_lights(const DevScene<R>& sc, F&& f) {
#ifdef RTC_JIT
    if constexpr (sizeof(R) == 4) {
        jit_light_each<0, jit::kNumLights>(f);
        return;
    }
#endif
    for (int li = 0; li < sc.n_lights; ++li) f(ld_uniform(&sc.lights[li]));
}

// calculate_lighting (material.rs:83-114) of one light: ambient always;
// diffuse and specular where the light is in front of the surface
// (ldn = light . normal >= 0) and the point is not shadowed.
template <typename R>
__device__ inline V3<R> lighting_term(const LightRec<R>& L, const MaterialRec<R>& m, V3<R> base, V3<R> n, V3<R> eye,
                                      V3<R> ld, R ldn, bool shadowed) {
    const V3<R> eff = {base.x * L.intensity[0], base.y * L.intensity[1], base.z * L.intensity[2]};
    V3<R> c = {eff.x * m.ambient, eff.y * m.ambient, eff.z * m.ambient};
    if (!shadowed) {
        if (!(ldn < (R)0)) {
            c = {c.x + (eff.x * m.diffuse) * ldn, c.y + (eff.y * m.diffuse) * ldn, c.z + (eff.z * m.diffuse) * ldn};
            const R rde = dot(reflect(vneg(ld), n), eye);
            // specular 0 (every wall of three_sphere) adds exactly +0: skip the
            // pow (two transcendentals) for those lanes
            if (!(rde <= (R)0) && m.specular != (R)0) {
                const R f = Real<R>::pow(rde, m.shininess);
                c = {c.x + (L.intensity[0] * m.specular) * f, c.y + (L.intensity[1] * m.specular) * f,
                     c.z + (L.intensity[2] * m.specular) * f};
            }
        }
    }
    return c;
}

template <typename R, bool kChildren, bool kDup = false, typename Push = NoPush>
__device__ inline bool shade_ray(const DevScene<R>& sc, V3<R> o, V3<R> d, uint32_t remaining, Shaded<R>& out,
                                 Push&& push = Push{}) {
    using T = Real<R>;
    const Hit<R> h = closest_hit(sc, o, d);
    if (h.slot < 0) return false;  // world.rs:85: miss -> BLACK
    Prepared<R> q;
#ifdef RTC_JIT
    MaterialRec<R> m_const;
    const MaterialRec<R>* mp;
    if constexpr (kJitConstMaterials && !kChildren && sizeof(R) == 4) {
        prepare_hit_const(sc, o, d, h, q, out.patterned, m_const);
        mp = &m_const;
    } else {
        mp = &prepare_hit(sc, o, d, h, q, out.patterned);
    }
    const MaterialRec<R>& m = *mp;
#else
    const MaterialRec<R>& m = prepare_hit(sc, o, d, h, q, out.patterned);
#endif
    const V3<R> p = q.p, n = q.n, eye = q.eye, over = q.over, base = q.base;
    const R off = q.off;
    V3<R> surface = {(R)0, (R)0, (R)0};
    for_lights(sc, [&](const LightRec<R>& L) {
        const V3<R> lpos = {L.position[0], L.position[1], L.position[2]};
        const V3<R> to_light = vsub(lpos, over);
        const R dist = magnitude(to_light);
        const V3<R> ld = normalized(to_light);  // == to_light / dist (world.rs:104-106)
        // calculate_lighting, material.rs:83-114.  The shadow test only
        // matters where the light is in front of the surface (ldn < 0 gives
        // ambient only, shadowed or not), so only those lanes trace it; the
        // reference traces it for every light (world.rs:46-52) and the event
        // counters still count one shadow ray per light.
        const R ldn = dot(ld, n);
        bool shadowed = false;
        if (!(ldn < (R)0) || !skips_on(sc)) shadowed = any_hit(sc, over, ld, dist, lpos);
        const V3<R> c = lighting_term(L, m, base, n, eye, ld, ldn, shadowed);
        surface = {surface.x + c.x, surface.y + c.y, surface.z + c.z};
    });
    out.surface = surface;
    out.refl_child = out.refr_child = false;
    // shade_hit evaluates Schlick whenever the material is both (world.rs:59-60)
    out.schlick = (m.reflectiveness > (R)0) & (m.transparency > (R)0);
    if constexpr (kChildren) {
#ifdef RTC_JIT
        constexpr bool kTransparent = jit::kTransparent;  // per-scene build: no glass, no refraction code
#else
        constexpr bool kTransparent = true;
#endif
        const bool reflective = m.reflectiveness > (R)0, transparent = kTransparent && m.transparency > (R)0;
        // n1 / n2 (the containers walk) feed only the children's weights and
        // the refracted direction, and a ray at remaining 0 has no children
        // (world.rs:120, 136): the walk runs for rays that can spawn.  (The
        // reference computes them in every prepare_computations; the values are
        // unused there too.)  The deepest generation is the largest one of a
        // glass tree, so this skips most walks: DESIGN.md §3.2.
        R n1 = (R)1, n2 = (R)1;
        if (kTransparent && m.transparency != (R)0 && remaining > 0)
            refractive_indices<R, kDup>(sc, o, d, h, q.mat, n1, n2);
        // Schlick mixing only when both (world.rs:59-66)
        R fr = (R)1, ft = (R)1;
        if (reflective && transparent) {  // computed_hit.rs:50-68
            R cs = dot(eye, n);
            bool total = false;
            if (n1 > n2) {
                const R ratio = T::div(n1, n2);
                const R sin2 = (ratio * ratio) * ((R)1 - cs * cs);
                if (sin2 > (R)1) total = true;
                else cs = T::sqrt((R)1 - sin2);
            }
            R rr = (R)1;
            if (!total) {
                const R q = T::div(n1 - n2, n1 + n2);
                const R r0 = q * q;
                const R x = (R)1 - cs;
                rr = T::rfma((R)1 - r0, x * ((x * x) * (x * x)), r0);
            }
            fr = rr;
            ft = (R)1 - rr;
        }
        if (remaining > 0 && m.reflectiveness != (R)0) {  // world.rs:114-128
            out.refl_child = true;
            push(over, reflect(d, n), m.reflectiveness * fr);
        }
        if (kTransparent && remaining > 0 && m.transparency != (R)0) {  // world.rs:130-157
            out.refr_eval = true;
            const R nr = T::div(n1, n2);
            const R cos_i = dot(eye, n);
            const R sin2_t = (nr * nr) * ((R)1 - cos_i * cos_i);
            if (!(sin2_t > (R)1)) {
                const R cos_t = T::sqrt((R)1 - sin2_t);
                const R f = T::rfma(nr, cos_i, -cos_t);
                out.refr_child = true;
                push(along(p, n, -off),  // under_point, computed_hit.rs:34
                     V3<R>{n.x * f - eye.x * nr, n.y * f - eye.y * nr, n.z * f - eye.z * nr}, m.transparency * ft);
            }
        }
    }
    return true;
}

// camera.rs:52-68
template <typename R>
__device__ inline void camera_ray(const CameraRec<R>& c, uint32_t x, uint32_t y, V3<R>& o, V3<R>& d) {
    const R ox = ((R)x + (R)0.5) * c.pixel_size;
    const R oy = ((R)y + (R)0.5) * c.pixel_size;
    const R wx = c.half_width - ox;
    const R wy = c.half_height - oy;
    o = {c.origin[0], c.origin[1], c.origin[2]};
    if constexpr (sizeof(R) == 4) {
        // pixel - origin == M3 * (wx, wy, -1): skip the cancelling translation
        d = normalized(xform_vector(c.inv, V3<R>{wx, wy, (R)-1}));
    } else {
        const V3<R> pixel = xform_point(c.inv, V3<R>{wx, wy, (R)-1});
        d = normalized(vsub(pixel, o));
    }
}

template <typename R>
__device__ inline void store_pixel(const LaunchParams<R>& P, uint64_t idx, V3<R> c) {
    if (P.out_format == RT_OUT_U8) {
        // canvas.rs:117-123: round(clamp(c, 0, 1) * 255), NaN -> 0
        auto q = [](R v) -> uint8_t {
            if (!(v == v)) return 0;
            v = v < (R)0 ? (R)0 : (v > (R)1 ? (R)1 : v);
            if constexpr (sizeof(R) == 4) return (uint8_t)__builtin_roundf(v * (R)255);
            else return (uint8_t)__builtin_round(v * (R)255);
        };
        uint8_t* o = static_cast<uint8_t*>(P.out) + 3 * idx;
        __builtin_nontemporal_store(q(c.x), o);
        __builtin_nontemporal_store(q(c.y), o + 1);
        __builtin_nontemporal_store(q(c.z), o + 2);
    } else {
        R* o = static_cast<R*>(P.out) + 3 * idx;
        __builtin_nontemporal_store(c.x, o);
        __builtin_nontemporal_store(c.y, o + 1);
        __builtin_nontemporal_store(c.z, o + 2);
    }
}

// Tile t of this launch -> pixel of thread `tid` (x, y, output index).
#ifndef RTC_WAVE_W
#define RTC_WAVE_W 16  // a wave's pixel block: 16 x 4 (64: one 64-pixel row)
#endif
static_assert(RT_TILE_W % RTC_WAVE_W == 0 && RT_TILE_H % (64 / RTC_WAVE_W) == 0, "the 4 waves tile the tile");
template <typename R>
__device__ inline bool tile_pixel(const LaunchParams<R>& P, uint32_t t, uint32_t tid, uint32_t& x, uint32_t& y,
                                  uint64_t& out_idx) {
    const uint32_t lrow = div_by(t, P.tiles_x, P.tiles_x_magic), tcol = t - lrow * P.tiles_x;
    // wave w of the tile covers one RTC_WAVE_W x (64 / RTC_WAVE_W) pixel block
    constexpr uint32_t kPerRow = RT_TILE_W / RTC_WAVE_W, kWaveH = 64 / RTC_WAVE_W;
    const uint32_t wave = tid / 64, lane = tid % 64;
    const uint32_t local_y = lrow * RT_TILE_H + (wave / kPerRow) * kWaveH + lane / RTC_WAVE_W;  // row in the strip
    x = tcol * RT_TILE_W + (wave % kPerRow) * RTC_WAVE_W + lane % RTC_WAVE_W;
    y = shard_image_row(local_y, P.shard_count, P.shard_index);
    out_idx = (uint64_t)(P.image_rows ? y : local_y) * P.width + x;
    return x < P.width && y < P.height;
}

// kFramesOnly: the caller never runs in color_at mode (per-scene direct
// kernels, rtc_host.cpp launch: camera frames only).  Same-box A/B: three_sphere
// 1080p 19.9 -> 19.4 us, shadow_puppets -1.6 %; the per-scene pool kernel
// lost 1-2 % that way (register allocation) and keeps the branch.
template <typename R, bool kFramesOnly = false>
__device__ inline void load_primary(const LaunchParams<R>& P, uint32_t t, uint32_t tid, bool& valid, V3<R>& o,
                                    V3<R>& d, uint64_t& out_idx) {
    if (!kFramesOnly && P.rays) {  // color_at mode: tile = 256 consecutive rays
        const uint64_t r = (uint64_t)t * kBlock + tid;
        valid = r < P.n_rays;
        out_idx = r;
        if (valid) {
            const double* q = P.rays + 6 * r;
            o = {(R)q[0], (R)q[1], (R)q[2]};
            d = {(R)q[3], (R)q[4], (R)q[5]};
        }
    } else {
        uint32_t x, y;
        valid = tile_pixel(P, t, tid, x, y, out_idx);
        if (valid) camera_ray(P.cam, x, y, o, d);
    }
}

// The workgroup's counters into its counter shard: each wave's lane 0 puts
// the wave's (uniform) counts in LDS, and after one barrier lanes 0..7 of
// wave 0 add the workgroup's sums, one atomic each.  (Every wave adding its
// own eight, one after another, cost 0.8 us of a 23.6 us three_sphere frame:
// the last waves' atomics sit on the kernel's tail.)  Called by every thread
// of the workgroup.
__device__ inline void flush_counts(const Counts& k, unsigned long long* global) {
    __shared__ uint32_t s_counts[kBlock / 64][kNumCounters];
    const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    if (lane == 0)
        for (int i = 0; i < kNumCounters; ++i) s_counts[wave][i] = k.c[i];
    __syncthreads();
    if (threadIdx.x < (uint32_t)kNumCounters) {
        unsigned long long v = 0;
        for (uint32_t w = 0; w < kBlock / 64; ++w) v += s_counts[w][threadIdx.x];
        const uint32_t shard = blockIdx.x % kCounterShards;
        if (v) atomicAdd(&global[shard * kNumCounters + threadIdx.x], v);
    }
}

// Next work item of this workgroup (called by thread 0 only; `probe` lives in
// its registers).  kSchedGrid: one workgroup per tile; kSchedStatic: tiles
// b, b+G, b+2G, ... of a resident grid, no atomics; kSchedDynamic: per-XCD
// queues, queue q holding tiles q, q+8, ....  A workgroup drains queue
// b % 8 (its XCD's under round-robin dispatch) and then steals from the
// others in turn: without stealing, a queue whose tiles were cheap left its
// XCD idle while another XCD's queue ran 300-450 us longer (reflect_refract,
// per-workgroup timestamps).  Every launch finds its heads zeroed (context
// creation, then the previous dynamic launch: trace_pool), so their atomics
// need no other bookkeeping.
template <typename R>
__device__ inline unsigned int next_tile(const LaunchParams<R>& P, uint32_t it, uint32_t& probe, uint32_t n_items) {
    if (P.persistent == kSchedGrid) return it == 0 ? blockIdx.x : kNoItem;
    if (P.persistent == kSchedStatic) {
        const unsigned long long t = blockIdx.x + (unsigned long long)it * gridDim.x;
        return t < P.n_tiles ? (unsigned int)t : kNoItem;
    }
    for (; probe < (uint32_t)kTileQueues; ++probe) {
        const uint32_t q = (blockIdx.x + probe) % kTileQueues;
        const unsigned long long j = atomicAdd(&P.tile_counter[q * kQueueStride], 1ull);
        const unsigned long long i = q + (unsigned long long)kTileQueues * j;
        if (i < n_items) return P.tile_order ? P.tile_order[i] : (unsigned int)i;
    }
    return kNoItem;
}

// The world as seen by one launch, rebuilt from the restrict parameters.
// With kLds the shape/material/pattern tables are first copied into the
// front of dynamic LDS (P.world_lds bytes, 16-byte words, one barrier) so
// the per-lane gathers of shade_ray are ds_reads rather than divergent
// global loads; the wave-uniform loops keep reading the global tables
// through the scalar cache.
template <typename R, bool kLds>
__device__ inline DevScene<R> scene_view(const LaunchParams<R>& P, const ShapeRec<R>* __restrict__ shapes,
                                         const MaterialRec<R>* __restrict__ materials,
                                         const PatternRec<R>* __restrict__ patterns,
                                         const LightRec<R>* __restrict__ lights, unsigned char* smem,
                                         bool stage = false) {
    DevScene<R> sc = P.scene;
    sc.no_skips = (P.flags & RT_FLAG_NO_SKIPS) != 0;
    sc.shapes = shapes;
    sc.materials = materials;
    sc.patterns = patterns;
    sc.lights = lights;
    if constexpr (kLds && kJitRecords && sizeof(R) == 4) {
        // per-scene records: only [materials][patterns] in LDS (no shapes, no world_slot)
        auto* lm = reinterpret_cast<MaterialRec<R>*>(smem);
        auto* lp = reinterpret_cast<PatternRec<R>*>(lm + sc.n_materials);
        if (stage) {
            const uint4* s4 = reinterpret_cast<const uint4*>(materials);  // followed by the patterns (DeviceWorld)
            uint4* d4 = reinterpret_cast<uint4*>(lm);
            for (uint32_t i = threadIdx.x; i < P.world_lds / 16; i += kBlock) d4[i] = s4[i];
            __syncthreads();
        }
        sc.lshapes = shapes;
        sc.lmats = lm;
        sc.lpats = lp;
        sc.lworld_slot = sc.world_slot;
    } else if constexpr (kLds) {
        const int ns = sc.kind_begin[kNumKinds];
        auto* ls = reinterpret_cast<ShapeRec<R>*>(smem);
        auto* lm = reinterpret_cast<MaterialRec<R>*>(ls + ns);
        auto* lp = reinterpret_cast<PatternRec<R>*>(lm + sc.n_materials);
        auto* lw = reinterpret_cast<int32_t*>(lp + sc.n_patterns);
        if (stage) {
            // The four tables are one allocation in this very layout
            // (rtc_context.hpp DeviceWorld), starting at `shapes`: one
            // contiguous copy, all loads in flight before the first LDS
            // write (four table-by-table loops waited on four load
            // latencies, in every one of the direct kernel's 5120 workgroups).
            const uint4* s4 = reinterpret_cast<const uint4*>(shapes);
            uint4* d4 = reinterpret_cast<uint4*>(ls);
            for (uint32_t i = threadIdx.x; i < P.world_lds / 16; i += kBlock) d4[i] = s4[i];
            __syncthreads();
        }
        sc.lworld_slot = lw;
        sc.lshapes = ls;
        sc.lmats = lm;
        sc.lpats = lp;
    } else {
        sc.lshapes = shapes;
        sc.lmats = materials;
        sc.lpats = patterns;
        sc.lworld_slot = sc.world_slot;
    }
    return sc;
}

// The launch's parameters re-read from the kernarg segment (the kernel's
// first explicit argument starts it).  The asm makes the pointer opaque, so
// loads through it cannot be hoisted out of the tile loop: scene counts,
// camera and canvas fields come back as s_loads (scalar cache) where they
// are used instead of being held in SGPRs for the whole kernel, which spilled
// ~60 of them into VGPR lanes (v_writelane/v_readlane: VALU issue slots).
template <typename R>
__device__ inline const LaunchParams<R>& kernarg_params() {
    auto k = __builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    return *(const LaunchParams<R>*)k;  // address-space cast (constant -> generic)
}

#define RTC_WORLD_PARAMS(R)                                                                                  \
    const ShapeRec<R>* __restrict__ shapes, const MaterialRec<R>* __restrict__ materials,                   \
        const PatternRec<R>* __restrict__ patterns, const LightRec<R>* __restrict__ lights

// --------------------------------------------------------------- kernels
// Waves per SIMD the f32 direct kernel is register-limited to (VGPRs <= 512 /
// waves).  Measured on MI355X, three_sphere 1080p (scripts/ab_builds.sh):
// 7 (<= 72 VGPRs) 46.0 us, unconstrained (74 VGPRs, 6 waves) 46.5 us,
// 8 (<= 64 VGPRs, spills at tile level) 48.9 us, with SLP vectorization on.
// Built without it (Makefile) the kernel needs 55 VGPRs, so 8 waves fit
// without spills: 34.5 us against 34.7 us at 7 waves with SLP.
#ifndef RTC_DIRECT_WAVES
#define RTC_DIRECT_WAVES 8
#endif
// Waves per SIMD of the f32 pool kernel (VGPRs <= 512 / waves; its LDS pool
// is sized to match, rtc_host.cpp pool_lds_rays).  Occupancy beats spills
// here: same-box A/B (scripts/ab_builds.sh), kernel time vs 4 waves (111
// VGPRs): 6 waves (80 VGPRs, 108 B/lane scratch) cover -11%, metal -7%,
// reflect_refract/table/refraction -4..-6%, cylinders +4%; 7 and 8 waves
// spill more and lose.  Without a cap a code change that crosses 128 VGPRs
// drops to 3 waves (~60% slower, measured).  Per-scene builds are also made
// at 7 (rtc_jit.cpp jit_function, jit_options.hpp) and kept where they spill
// little: reflect_refract, table and cover run at 7 since round 5.
#ifndef RTC_POOL_WAVES
#define RTC_POOL_WAVES 6
#endif
template <typename R, bool kLds>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(sizeof(R) == 4 ? RTC_DIRECT_WAVES : 1))) void trace_direct(
    LaunchParams<R> P, RTC_WORLD_PARAMS(R)) {
    extern __shared__ __align__(16) unsigned char smem[];
    (void)scene_view<R, kLds>(P, shapes, materials, patterns, lights, smem, true);
#ifdef RTC_JIT
    // per-scene builds run no diagnostics (RT_FLAG_STAMPS / NO_SHADE / NO_TRACE
    // launches take the generic kernel, rtc_host.cpp launch)
    constexpr bool kDiag = false;
#else
    const bool kDiag = true;
#endif
    if (kDiag && P.stamps && threadIdx.x == 0) P.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    Counts k = {};
    const uint32_t tid = threadIdx.x;
    // Tiles b, b+G, b+2G, ...: with G = n_tiles (kSchedGrid) one tile per
    // workgroup, with G = resident workgroups (kSchedStatic) a persistent
    // grid.  Primary-only tiles cost the same, so no queue is needed, and the
    // tile index is an SGPR by construction (loop control stays scalar).
    for (uint32_t t = blockIdx.x;; t += gridDim.x) {
        const LaunchParams<R>& P = kernarg_params<R>();
        const DevScene<R> sc = scene_view<R, kLds>(P, shapes, materials, patterns, lights, smem);
        if (t >= P.n_tiles) break;
        bool valid;
        V3<R> o, d;
        uint64_t out_idx;
#ifdef RTC_JIT
        load_primary<R, true>(P, t, tid, valid, o, d, out_idx);
#else
        load_primary(P, t, tid, valid, o, d, out_idx);
#endif
        V3<R> c = {(R)0, (R)0, (R)0};
        Shaded<R> sh;
        bool hit = false;
        if (valid) {
            if (kDiag && (P.flags & (RT_FLAG_NO_SHADE | RT_FLAG_NO_TRACE))) {
                if (P.flags & RT_FLAG_NO_TRACE) {
                    c = d;
                } else {
                    const Hit<R> h = closest_hit(sc, o, d);
                    c = {h.t * (R)0.01, (R)h.slot, (R)0};
                }
            } else if (shade_ray<R, false>(sc, o, d, 0, sh)) {
                hit = true;
                c = sh.surface;
            }
        }
        count_events(k, valid, hit, sh, sc.n_lights);
        if (kDiag && P.gen_counts) count_generations(P.gen_counts, valid, hit, P.max_depth);
        if (valid) store_pixel(P, out_idx, c);
    }
    if (!(P.flags & RT_FLAG_NO_COUNTERS)) flush_counts(k, P.counters);
    if (kDiag && P.stamps) {
        __syncthreads();
        if (threadIdx.x == 0) P.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// s_setprio takes an immediate.
__device__ inline void set_wave_prio(uint32_t p) {
    if (p == 0) __builtin_amdgcn_s_setprio(0);
    else if (p == 1) __builtin_amdgcn_s_setprio(1);
    else if (p == 2) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(3);
}

// Ray pool: one LIFO of pending rays per WORKGROUP, run in block-lockstep
// generations (trace_pool).  Dynamic LDS after the world tables holds
//   [acc: kTileSlots (1) x 3 x kBlock PoolAcc<R>: the tile's pixel sums]
//   [ox oy oz dx dy dz w : lds_cap x R][meta : lds_cap x PoolMeta]
// with meta = pixel | remaining << 8 (pixel = the lane of the 64x4 tile,
// 0..255; 13 bits, so 16-bit entries give the pool 1/16 more slots in the
// same LDS; rtc_internal.hpp PoolMeta).  Slots [lds_cap, cap) live in the
// workgroup's region of P.spill, one 8-word record per entry (AoS: a lane's
// entry is two dwordx4 stores / loads in f32, where the SoA layout took
// eight dword instructions per entry; the record keeps meta in 32 bits).
// The LIFO bound cap = kBlock + depth x batch (rtc_host.cpp pool_capacity)
// makes overflow impossible; the LDS part is sized for occupancy
// (plan_launch), deep excursions spill.
template <typename R>
struct Pool {
    PoolAcc<R>* acc;
    R* lds;    // 8 arrays of lds_cap words: ox oy oz dx dy dz w, then meta (u32)
    R* spill;  // spill_cap records of 8 words (this workgroup's region)
    int lds_cap, spill_cap;
#ifdef RTC_BOUNDS_CHECK
    int32_t* err;  // LaunchParams::error_flag
#endif
};

// RTC_BOUNDS_CHECK (debug builds): false, with the bit raised, when an index
// is outside its buffer; the caller then skips the access.  Product builds
// compile the checks out.
__device__ inline bool in_bounds(bool ok, int32_t* err, int32_t bit) {
#ifdef RTC_BOUNDS_CHECK
    if (!ok) atomicOr(err, bit);
    return ok;
#else
    (void)err;
    (void)bit;
    (void)ok;
    return true;
#endif
}

// Reserve `pred` slots for the lanes of one wave: ballot + mbcnt prefix, one
// LDS atomic per wave.  Returns the lane's slot or -1.
__device__ inline int wave_reserve(bool pred, int* top) {
    const unsigned long long m = __builtin_amdgcn_ballot_w64(pred);
    if (m == 0) return -1;
    const int prefix = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(top, __popcll(m));
    base = __shfl(base, leader);
    return pred ? base + prefix : -1;
}

// One base pointer and a stride per level (not 16 pointers: those were
// kept in VGPRs and spilled to scratch), and one branch per level so each
// side keeps its address space (ds_* for LDS, global_* for the spill; a
// pointer that may be either becomes flat_*).  meta = pixel | remaining << 8.
#define RTC_AS_LDS __attribute__((address_space(3)))
#define RTC_AS_GLOBAL __attribute__((address_space(1)))

template <typename R, typename PR, typename PU>
__device__ inline void pool_store(PR base, PU metas, int n, int i, V3<R> o, V3<R> d, R w, uint32_t meta) {
    base[i] = o.x;
    base[n + i] = o.y;
    base[2 * n + i] = o.z;
    base[3 * n + i] = d.x;
    base[4 * n + i] = d.y;
    base[5 * n + i] = d.z;
    base[6 * n + i] = w;
    metas[i] = meta;
}

template <typename R, typename PR, typename PU>
__device__ inline void pool_load(PR base, PU metas, int n, int i, V3<R>& o, V3<R>& d, R& w, uint32_t& meta) {
    o = {base[i], base[n + i], base[2 * n + i]};
    d = {base[3 * n + i], base[4 * n + i], base[5 * n + i]};
    w = base[6 * n + i];
    meta = metas[i];
}

// A spilled entry: {o.x, o.y, o.z, d.x} {d.y, d.z, w, meta bits} (f32: two
// 16-byte vector accesses; f64: four).  The meta word travels as raw bits.
template <typename R>
__device__ inline void spill_store(RTC_AS_GLOBAL R* e, V3<R> o, V3<R> d, R w, uint32_t meta) {
    if constexpr (sizeof(R) == 4) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        RTC_AS_GLOBAL f4* p = (RTC_AS_GLOBAL f4*)e;
        p[0] = f4{o.x, o.y, o.z, d.x};
        p[1] = f4{d.y, d.z, w, __uint_as_float(meta)};
    } else {
        typedef double d2 __attribute__((ext_vector_type(2)));
        RTC_AS_GLOBAL d2* p = (RTC_AS_GLOBAL d2*)e;
        p[0] = d2{o.x, o.y};
        p[1] = d2{o.z, d.x};
        p[2] = d2{d.y, d.z};
        p[3] = d2{w, __longlong_as_double((long long)meta)};
    }
}

template <typename R>
__device__ inline void spill_load(const RTC_AS_GLOBAL R* e, V3<R>& o, V3<R>& d, R& w, uint32_t& meta) {
    if constexpr (sizeof(R) == 4) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const RTC_AS_GLOBAL f4* p = (const RTC_AS_GLOBAL f4*)e;
        const f4 a = p[0], b = p[1];
        o = {a.x, a.y, a.z};
        d = {a.w, b.x, b.y};
        w = b.z;
        meta = __float_as_uint(b.w);
    } else {
        typedef double d2 __attribute__((ext_vector_type(2)));
        const RTC_AS_GLOBAL d2* p = (const RTC_AS_GLOBAL d2*)e;
        const d2 a = p[0], b = p[1], c = p[2], q = p[3];
        o = {a.x, a.y, b.x};
        d = {b.y, c.x, c.y};
        w = q.x;
        meta = (uint32_t)__double_as_longlong(q.y);
    }
}

template <typename R>
__device__ inline void pool_put(const Pool<R>& pl, int slot, V3<R> o, V3<R> d, R w, uint32_t meta) {
#ifdef RTC_BOUNDS_CHECK
    if (!in_bounds(slot >= 0 && slot < pl.lds_cap + pl.spill_cap, pl.err, kErrBoundsSlot)) return;
#endif
    if (slot < pl.lds_cap) {
        RTC_AS_LDS R* b = (RTC_AS_LDS R*)pl.lds;
        pool_store<R>(b, (RTC_AS_LDS PoolMeta*)(b + 7 * pl.lds_cap), pl.lds_cap, slot, o, d, w, meta);
    } else {
        spill_store<R>((RTC_AS_GLOBAL R*)pl.spill + 8 * (size_t)(slot - pl.lds_cap), o, d, w, meta);
    }
}

template <typename R>
__device__ inline void pool_get(const Pool<R>& pl, int slot, V3<R>& o, V3<R>& d, R& w, uint32_t& meta) {
#ifdef RTC_BOUNDS_CHECK
    if (!in_bounds(slot >= 0 && slot < pl.lds_cap + pl.spill_cap, pl.err, kErrBoundsSlot)) {
        o = d = {(R)0, (R)0, (R)0};
        w = (R)0;
        meta = 0;
        return;
    }
#endif
    if (slot < pl.lds_cap) {
        const RTC_AS_LDS R* b = (const RTC_AS_LDS R*)pl.lds;
        pool_load<R>(b, (const RTC_AS_LDS PoolMeta*)(b + 7 * pl.lds_cap), pl.lds_cap, slot, o, d, w, meta);
    } else {
        spill_load<R>((const RTC_AS_GLOBAL R*)pl.spill + 8 * (size_t)(slot - pl.lds_cap), o, d, w, meta);
    }
}

// One contribution w x surface into pixel `pix`'s fixed-point sum (an LDS
// atomic: the sum does not depend on the order waves add in).  f64: int64
// multiples of 2^-48.  f32: int32 multiples of 2^-acc_log2 (the launch's
// scale, sized to the world's brightness bound by the host, acc_shift_f32):
// v x 2^s is exact in f32 and rounds to the nearest integer once.
__device__ inline void acc_add(long long* acc, uint32_t pix, double v, float) {
    const long long q = __double2ll_rn(v * kAccScale);
    if (q) atomicAdd(reinterpret_cast<unsigned long long*>(&acc[pix]), (unsigned long long)q);
}
__device__ inline void acc_add(int* acc, uint32_t pix, float v, float scale) {
    const int q = (int)__builtin_rintf(v * scale);
    if (q) atomicAdd(&acc[pix], q);
}

// The output element of thread `tid` of tile t (a pixel of a frame, or ray
// t * kBlock + tid of a color_at batch); false outside the canvas / batch.
template <typename R>
__device__ inline bool item_pixel(const LaunchParams<R>& P, uint32_t t, uint32_t tid, uint64_t& out_idx) {
    if (P.rays) {
        const uint64_t r = (uint64_t)t * kBlock + tid;
        out_idx = r;
        return r < P.n_rays;
    }
    uint32_t x, y;
    return tile_pixel(P, t, tid, x, y, out_idx);
}

// trace_pool: the recursion as a per-workgroup LIFO ray pool run in
// block-lockstep generations.  The round-5 free-running
// variant that dropped the per-generation barriers (slower, §3.2) is kept
// out of the product source as scripts/patches/pool_free_and_diag.patch.
template <typename R, bool kLds, bool kDup>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(sizeof(R) == 4 ? RTC_POOL_WAVES : 1))) void trace_pool(
    LaunchParams<R> P, RTC_WORLD_PARAMS(R)) {
    extern __shared__ __align__(16) unsigned char smem_all[];
    const DevScene<R> sc = scene_view<R, kLds>(P, shapes, materials, patterns, lights, smem_all, true);
    // (per-scene pool builds keep the diagnostics: same-box A/B without them
    // reflect_refract, refraction, metal within 1 %)
    constexpr bool kDiag = true;
    if (kDiag && P.stamps && threadIdx.x == 0) P.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    unsigned char* smem = smem_all + (kLds ? P.world_lds : 0);
    __shared__ unsigned int s_tile[2];
    __shared__ int s_top[2];
    const uint32_t cap = P.pool_capacity;
    const uint32_t lcap = P.pool_lds_capacity, gcap = cap - lcap;
    Pool<R> pl;
    pl.acc = reinterpret_cast<PoolAcc<R>*>(smem);
    pl.lds = reinterpret_cast<R*>(smem + 3 * kBlock * sizeof(PoolAcc<R>));
    const float acc_scale = __builtin_ldexpf(1.0f, (int)P.acc_log2);
    pl.lds_cap = (int)lcap;
    // 8 words per spilled entry; blockIdx.x < grid (persistent launch)
    pl.spill = reinterpret_cast<R*>(P.spill) + spill_word(blockIdx.x, gcap, lcap, lcap);
    pl.spill_cap = (int)gcap;
#ifdef RTC_BOUNDS_CHECK
    pl.err = P.error_flag;
    if (!in_bounds(gcap == 0 || blockIdx.x < P.spill_blocks, P.error_flag, kErrBoundsSpill)) pl.spill_cap = 0;
#endif

    Counts k = {};
    const uint32_t tid = threadIdx.x;
    // Two sets of queue heads alternate between dynamic launches: this launch
    // zeroes the set the next one uses (its last user, the previous launch,
    // has completed: stream order).
    if (P.persistent == kSchedDynamic && blockIdx.x == 0 && tid < (uint32_t)kTileQueues)
        P.next_tile_counter[tid * kQueueStride] = 0ull;
    uint32_t probe = 0;
    // thread 0: the items of this launch (read once: it sits on the dequeue path)
    const uint32_t n_items = P.item_count && tid == 0 ? *P.item_count : P.n_tiles;
    unsigned long long tile_start = 0;  // thread 0: s_memrealtime at the tile's start
    for (uint32_t it = 0;; ++it) {
        if (tid == 0) {
            s_tile[it & 1] = next_tile(P, it, probe, n_items);
            s_top[0] = 0;
            tile_start = __builtin_amdgcn_s_memrealtime();
        }
        for (int c = 0; c < 3; ++c) pl.acc[c * kBlock + tid] = 0;
        __syncthreads();
        const uint32_t item = __builtin_amdgcn_readfirstlane(s_tile[it & 1]);
        if (item == kNoItem) break;
        // packed fields only in items handed out through a tile order (raster
        // items are plain tile indices, any number of them)
        const WorkItem wi = decode_item(item, P.tile_order != nullptr);
        const uint32_t t = wi.tile, split = wi.split_log2;
#ifdef RTC_BOUNDS_CHECK
        if (!in_bounds(t < P.n_tiles, P.error_flag, kErrBoundsTile)) continue;  // (every thread: uniform)
#endif
        // the costliest items set the launch's tail: their waves win issue
        // arbitration against the other workgroups' on the same SIMDs
        const uint32_t prio = wi.prio;
        if (prio) set_wave_prio(prio);
        bool valid;
        V3<R> o, d;
        uint64_t out_idx;
        load_primary(P, t, tid, valid, o, d, out_idx);
        // this item's part of the tile (all of it unless split)
        valid &= item_seeds(tid, wi);
        k.c[0] += wave_count(valid);
        {
            const int slot = wave_reserve(valid, &s_top[0]);
            if (valid) pool_put(pl, slot, o, d, (R)1, tid | (P.max_depth << 8));
        }
        __syncthreads();
        for (uint32_t gen = 0;; ++gen) {
            const int cur = gen & 1;
            const int size = s_top[cur];
            if (size == 0) break;
            const int kpop = size < (int)P.pop_batch ? size : (int)P.pop_batch;
            const int bottom = size - kpop;
            const bool active = (int)tid < kpop;
            V3<R> ro, rd;
            R rw = (R)0;
            uint32_t meta = 0;
            if (active) pool_get(pl, bottom + (int)tid, ro, rd, rw, meta);
            if (tid == 0) s_top[cur ^ 1] = bottom;
            __syncthreads();  // every lane holds its ray; the next top is set
            Shaded<R> sh;
            bool hit = false;
            const uint32_t pix = meta & 0xFFu;
            const uint32_t child_meta = pix | (((meta >> 8) - 1u) << 8);
            // lanes spawning a child reserve pool slots together (ballot +
            // one LDS atomic per wave) at the point the child is made
            auto push = [&](V3<R> co, V3<R> cd, R cw) {
                const int slot = wave_reserve(true, &s_top[cur ^ 1]);
                if (slot < (int)cap) pool_put(pl, slot, co, cd, rw * cw, child_meta);
                else atomicOr(P.error_flag, kErrPoolOverflow);
            };
            if (active) hit = shade_ray<R, true, kDup>(sc, ro, rd, meta >> 8, sh, push);
            count_events(k, false, hit, sh, sc.n_lights);
#ifndef RTC_JIT  // (per-scene builds never take RT_FLAG_GENERATIONS launches)
            if (P.gen_counts) count_generations(P.gen_counts, active, hit, meta >> 8);
#endif
            if (hit) {
                acc_add(pl.acc, pix, sh.surface.x * rw, acc_scale);
                acc_add(pl.acc + kBlock, pix, sh.surface.y * rw, acc_scale);
                acc_add(pl.acc + 2 * kBlock, pix, sh.surface.z * rw, acc_scale);
            }
            __syncthreads();  // pushes complete before the next pop
            if (s_top[cur ^ 1] > (int)cap) {  // overflowed: drop the pool (error already flagged)
                __syncthreads();
                if (tid == 0) s_top[cur ^ 1] = 0;
                __syncthreads();
            }
        }
        const double inv = sizeof(PoolAcc<R>) == 4 ? __builtin_ldexp(1.0, -(int)P.acc_log2) : kAccInvScale;
        const V3<R> c = {(R)((double)pl.acc[tid] * inv), (R)((double)pl.acc[kBlock + tid] * inv),
                         (R)((double)pl.acc[2 * kBlock + tid] * inv)};
#ifdef RTC_BOUNDS_CHECK
        valid &= in_bounds(!valid || out_idx < (P.rays ? P.n_rays
                                                       : (uint64_t)(P.image_rows ? P.height : P.tile_rows * RT_TILE_H) *
                                                             P.width),
                           P.error_flag, kErrBoundsOut);
#endif
        if (valid) store_pixel(P, out_idx, c);
        if (prio) __builtin_amdgcn_s_setprio(0);
        __syncthreads();  // accumulators are re-zeroed for the next tile
        // this tile's cost (10 ns ticks) orders the next launch of the same
        // frame heaviest-first (order_tiles)
        // (a split tile: its slowest part times the parts, order_tiles zeroed it)
        if (tid == 0 && P.tile_cost) {
            const uint32_t c = (uint32_t)min(__builtin_amdgcn_s_memrealtime() - tile_start, 0x0FFFFFFFull);
            if (split) atomicMax(&P.tile_cost[t], c << split);
            else P.tile_cost[t] = c;
        }
        if (kDiag && tid == 0 && P.item_log) {  // diagnostics (RT_FLAG_STAMPS): the item's span
            const unsigned long long k = atomicAdd(&P.item_log[0], 1ull);
            P.item_log[1 + 3 * k] = item | (unsigned long long)blockIdx.x << 32;
            P.item_log[2 + 3 * k] = tile_start;
            P.item_log[3 + 3 * k] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (!(P.flags & RT_FLAG_NO_COUNTERS)) flush_counts(k, P.counters);
    if (kDiag && P.stamps) {
        __syncthreads();
        if (threadIdx.x == 0) P.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}


#ifndef RTC_PRECISION
#define RTC_PRECISION 0
#endif
#if !defined(RTC_JIT) && RTC_PRECISION != 2  // the per-scene build holds the tracer kernels only; helpers in the f32 TU
// Heaviest-first work order from the previous launch's per-tile costs: a
// one-workgroup bucket sort (8 buckets per octave of cost, descending).  The
// pool kernel's time is set by its last, heaviest tiles (a glass-sphere tile
// of reflect_refract runs ~400 us); handing those out first bounds the tail
// (longest-processing-time-first).  Order within a bucket is arbitrary:
// tiles are independent and pixel sums are fixed-point, so images are not
// affected.
//
// A tile costing more than split_factor x the mean workgroup load (sum of
// costs / grid) is handed out as 2, 4 (8 or 16: RTC_DEBUG=split_max=3, 4) parts (items, rtc_internal.hpp): when
// a launch has few tiles per workgroup (a shard of a multi-GPU frame) its
// heaviest tiles outlast everything else, and the parts of one run on
// different CUs.  The parts' seeds cover a quarter or half of the tile, and
// its rays fill the pool within a few generations.  Split tiles' costs are
// zeroed here and rebuilt by their parts (atomicMax of part cost x parts).
constexpr int kOrderBuckets = 256;
constexpr int kOrderThreads = 1024;

__device__ inline uint32_t cost_bucket(uint32_t c) {  // 0 = heaviest
    const uint32_t b = (uint32_t)(__builtin_amdgcn_logf((float)c + 1.0f) * 8.0f);
    return (uint32_t)(kOrderBuckets - 1) - (b < (uint32_t)kOrderBuckets ? b : (uint32_t)(kOrderBuckets - 1));
}

// log2 of the parts a tile of cost c is split into: the least l >= min_log2
// with c / 2^l <= limit, at most max_log2
__device__ inline uint32_t split_log2(uint32_t c, float limit, uint32_t max_log2, uint32_t min_log2) {
    uint32_t l = min_log2;
    while (l < max_log2 && (float)c > limit * (float)(1u << l)) ++l;
    return l;
}

__global__ __launch_bounds__(kOrderThreads) void order_tiles(uint32_t* __restrict__ cost,
                                                             uint32_t* __restrict__ order, uint32_t n,
                                                             uint32_t* __restrict__ n_items, float split_per_cost,
                                                             uint32_t max_log2, float urgent_per_cost,
                                                             uint32_t graded, uint32_t min_log2) {
    __shared__ uint32_t hist[kOrderBuckets];
    __shared__ uint32_t scan[kOrderBuckets];
    __shared__ unsigned long long total;
    __shared__ uint32_t items;
    for (uint32_t b = threadIdx.x; b < (uint32_t)kOrderBuckets; b += kOrderThreads) hist[b] = 0;
    if (threadIdx.x == 0) {
        total = 0;
        items = 0;
    }
    __syncthreads();
    // wave sums first: 1024 same-address LDS atomics serialized to ~8 us
    auto wave_sum = [](unsigned long long v) {
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        return v;
    };
    float limit = __FLT_MAX__, urgent = __FLT_MAX__;  // split nothing, nothing urgent
    if (split_per_cost > 0.0f || urgent_per_cost > 0.0f) {
        unsigned long long mine = 0;
        for (uint32_t i = threadIdx.x; i < n; i += kOrderThreads) mine += cost[i];
        mine = wave_sum(mine);
        if ((threadIdx.x & 63) == 0) atomicAdd(&total, mine);
        __syncthreads();
        if (split_per_cost > 0.0f) limit = (float)total * split_per_cost;
        if (urgent_per_cost > 0.0f) urgent = (float)total * urgent_per_cost;
    }
    unsigned long long mine_items = 0;
    for (uint32_t i = threadIdx.x; i < n; i += kOrderThreads) {
        const uint32_t c = cost[i], l = split_log2(c, limit, max_log2, min_log2);
        atomicAdd(&hist[cost_bucket(c >> l)], 1u << l);
        mine_items += 1u << l;
    }
    mine_items = wave_sum(mine_items);
    if ((threadIdx.x & 63) == 0) atomicAdd(&items, (uint32_t)mine_items);
    __syncthreads();
    // Exclusive scan of the 256 bucket counts: Hillis-Steele over LDS.
    const uint32_t t = threadIdx.x;
    uint32_t own = 0;
    if (t < (uint32_t)kOrderBuckets) {
        own = hist[t];
        scan[t] = own;
    }
    __syncthreads();
    for (uint32_t off = 1; off < (uint32_t)kOrderBuckets; off <<= 1) {
        uint32_t v = 0;
        if (t < (uint32_t)kOrderBuckets && t >= off) v = scan[t - off];
        __syncthreads();
        if (t < (uint32_t)kOrderBuckets) scan[t] += v;
        __syncthreads();
    }
    if (t < (uint32_t)kOrderBuckets) hist[t] = scan[t] - own;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += kOrderThreads) {
        const uint32_t c = cost[i], l = split_log2(c, limit, max_log2, min_log2);
        const uint32_t pos = atomicAdd(&hist[cost_bucket(c >> l)], 1u << l);
        // priority: 3 above the urgent cost, or graded 1/2/3 above 1x/2x/4x it
        const float pc = (float)(c >> l);
        const uint32_t pr = !(pc > urgent) ? 0u : !graded ? 3u : pc > 4.0f * urgent ? 3u : pc > 2.0f * urgent ? 2u : 1u;
        for (uint32_t p = 0; p < (1u << l); ++p) order[pos + p] = encode_item(i, p, l, pr);
        if (l) cost[i] = 0;
    }
    if (threadIdx.x == 0) *n_items = items;
}

// Peer canvas completion (rt_render_to_canvas / rt_canvas_wait).  A shard's
// pixels reach the canvas (local, or another GPU's through an IPC or peer
// mapping) from its render kernel; this one-thread kernel, stream-ordered
// after it, publishes flag = seq with a system-scope release (every earlier
// write of this device visible first), so the canvas owner can consume the
// frame once every shard's flag holds the frame's sequence number.
__global__ void canvas_signal(unsigned long long* flag, unsigned long long seq) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Lane i < n polls flag i (system-scope acquire) until it reaches seq, or
// until timeout_ticks of s_memrealtime (100 MHz) have passed, which raises
// kErrPeerTimeout: every lane leaves the loop either way, so the kernel
// always drains.  Stream-ordered before the canvas's consumers.
__global__ void canvas_wait(const unsigned long long* flags, uint32_t n, unsigned long long seq,
                            unsigned long long timeout_ticks, int32_t* err) {
    const uint32_t i = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool late = false;
    for (uint32_t f = i; f < n; f += blockDim.x) {
        while (__hip_atomic_load(&flags[f], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
                late = true;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    if (late) atomicOr(err, kErrPeerTimeout);
    __threadfence_system();
}

// De-interleave gathered shard strips into one image.
__global__ void assemble_shards(const unsigned char* __restrict__ gathered, unsigned char* __restrict__ image,
                                uint32_t width, uint32_t height, uint32_t shards, uint32_t strip_rows,
                                uint32_t bpp) {
    const uint64_t row_bytes = (uint64_t)width * bpp;
    const uint32_t y = blockIdx.y;
    if (y >= height) return;
    uint32_t shard, strip_row;
    shard_of_image_row(y, shards, &shard, &strip_row);
    const uint64_t src_row = (uint64_t)shard * strip_rows + strip_row;
    const unsigned char* src = gathered + src_row * row_bytes;
    unsigned char* dst = image + (uint64_t)y * row_bytes;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    if (((row_bytes | (uintptr_t)gathered | (uintptr_t)image) & 15) == 0) {
        // 16-byte rows (every width of an f32/f64 canvas, u8 ones of width
        // % 16 == 0: a 4K u8 frame): one dwordx4 per thread instead of 16
        // byte accesses (round 5: the 1-rank tiled cover 4K frame's gather +
        // de-interleave 62 -> 11 us with rank 0's in-place gather, rtc_group.cpp)
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < row_bytes / 16; i += stride)
            d4[i] = s4[i];
        return;
    }
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < row_bytes; i += stride) dst[i] = src[i];
}
#endif  // helper kernels
#ifndef RTC_JIT

// Known-answer harness (rt_debug_intersect / rt_debug_normal): the product's
// own per-shape device code on caller-given rays or points, so the
// reference's per-shape unit tests (sphere.rs, plane.rs, cube.rs, cylinder.rs,
// cone.rs, triangle.rs, ray.rs) run against the GPU.  mode 0: intersect
// (every entry the reference pushes, in push order; world_space transforms
// the ray by the shape's inverse first, ray.rs:45-49, else the ray is
// already local as in local_intersect); mode 1: normal (world_space:
// normal_at, shape.rs:22-27; else local_normal_at).
constexpr int kDebugMaxEntries = RT_DEBUG_MAX_ENTRIES;

template <typename R>
__global__ void debug_shape(const ShapeRec<R>* __restrict__ shapes, int slot, int kind, uint32_t mode,
                            uint32_t world_space, const double* __restrict__ in, uint32_t n,
                            double* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ShapeRec<R> s = shapes[slot];
    if (mode == 0) {
        const double* q = in + 6 * (size_t)i;
        V3<R> o = {(R)q[0], (R)q[1], (R)q[2]}, d = {(R)q[3], (R)q[4], (R)q[5]};
        double* r0 = out + (1 + kDebugMaxEntries) * (size_t)i;
        if (world_space && kind == RT_SHAPE_SPHERE && world_sphere<R, RT_SHAPE_SPHERE>(s)) {  // the tracers' own test
            int c = 0;
            const R dd = dot(d, d);
            sphere_world<R, false>(s, o, d, dd, recip(dd), [&](R t, bool v) {
                if (v && c < kDebugMaxEntries) r0[1 + c++] = (double)t;
            });
            r0[0] = (double)c;
            return;
        }
        if (world_space && kind == RT_SHAPE_CUBE && world_cube<R, RT_SHAPE_CUBE>(s)) {
            int c = 0;
            cube_world<R, false>(s, o, d, recip3(d), [&](R t, bool v) {
                if (v && c < kDebugMaxEntries) r0[1 + c++] = (double)t;
            });
            r0[0] = (double)c;
            return;
        }
        if (world_space) {
            const V3<R> lo = xform_point(s.inv, o), ld = xform_vector(s.inv, d);
            o = lo;
            d = ld;
        }
        double* r = out + (1 + kDebugMaxEntries) * (size_t)i;
        int c = 0;
        auto emit = [&](R t, bool v) {
            if (v && c < kDebugMaxEntries) r[1 + c++] = (double)t;
        };
        switch (kind) {
            case RT_SHAPE_SPHERE: entries<R, RT_SHAPE_SPHERE>(s, o, d, emit); break;
            case RT_SHAPE_PLANE: entries<R, RT_SHAPE_PLANE>(s, o, d, emit); break;
            case RT_SHAPE_CUBE: entries<R, RT_SHAPE_CUBE>(s, o, d, emit); break;
            case RT_SHAPE_CYLINDER: entries<R, RT_SHAPE_CYLINDER>(s, o, d, emit); break;
            case RT_SHAPE_CONE: entries<R, RT_SHAPE_CONE>(s, o, d, emit); break;
            default: entries<R, RT_SHAPE_TRIANGLE>(s, o, d, emit); break;
        }
        r[0] = (double)c;
    } else {
        const double* q = in + 3 * (size_t)i;
        const V3<R> p = {(R)q[0], (R)q[1], (R)q[2]};
        const V3<R> nv = world_space ? normal_at(s, kind, p) : local_normal(s, kind, p);
        out[3 * (size_t)i] = (double)nv.x;
        out[3 * (size_t)i + 1] = (double)nv.y;
        out[3 * (size_t)i + 2] = (double)nv.z;
    }
}

// ------------------------------------------------------------ launchers
template <typename R>
hipError_t launch_trace(const LaunchParams<R>& P, bool pool, bool dup, uint32_t grid, size_t dyn_lds,
                        hipStream_t stream) {
    // hipLaunchKernelGGL reports through hipGetLastError(): drop any stale
    // error first (every earlier call's own status is checked by the host).
    (void)hipGetLastError();
    const bool lds = P.world_lds != 0;
#define RTC_LAUNCH(K, ...)                                                                                \
    hipLaunchKernelGGL((K<R, __VA_ARGS__>), dim3(grid), dim3(kBlock), dyn_lds, stream, P, P.scene.shapes,         \
                       P.scene.materials, P.scene.patterns, P.scene.lights)
    if (pool) {
#ifdef RTC_VARIANT
        if (dup) return hipErrorInvalidValue;  // worlds with value-equal shapes use the all-kinds build
        if (lds) RTC_LAUNCH(trace_pool, true, false);
        else RTC_LAUNCH(trace_pool, false, false);
#else
        if (lds) {
            if (dup) RTC_LAUNCH(trace_pool, true, true);
            else RTC_LAUNCH(trace_pool, true, false);
        } else {
            if (dup) RTC_LAUNCH(trace_pool, false, true);
            else RTC_LAUNCH(trace_pool, false, false);
        }
#endif
    } else {
#ifdef RTC_VARIANT
        return hipErrorInvalidValue;  // kind variants hold the pool kernel only
#else
        if (lds) RTC_LAUNCH(trace_direct, true);
        else RTC_LAUNCH(trace_direct, false);
#endif
    }
#undef RTC_LAUNCH
    return hipGetLastError();
}

template <typename R>
hipError_t occupancy(bool pool, bool lds, size_t dyn_lds, int* blocks_per_cu) {
    if (pool)
        return lds ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, trace_pool<R, true, false>, kBlock,
                                                                  dyn_lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, trace_pool<R, false, false>, kBlock,
                                                                  dyn_lds);
#ifdef RTC_VARIANT
    return hipErrorInvalidValue;
#endif
    return lds ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, trace_direct<R, true>, kBlock, dyn_lds)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, trace_direct<R, false>, kBlock, dyn_lds);
}

#if RTC_PRECISION != 2
template hipError_t launch_trace<float>(const LaunchParams<float>&, bool, bool, uint32_t, size_t, hipStream_t);
template hipError_t occupancy<float>(bool, bool, size_t, int*);
#endif
#ifndef RTC_VARIANT
#if RTC_PRECISION != 1
template hipError_t launch_trace<double>(const LaunchParams<double>&, bool, bool, uint32_t, size_t, hipStream_t);
template hipError_t occupancy<double>(bool, bool, size_t, int*);
#endif

#if RTC_PRECISION != 2
hipError_t launch_order_tiles(uint32_t* cost, uint32_t* order, uint32_t n, uint32_t* n_items, float split_per_cost,
                              uint32_t max_split_log2, float urgent_per_cost, uint32_t graded, uint32_t min_split_log2,
                              hipStream_t stream) {
    (void)hipGetLastError();  // see launch_trace
    hipLaunchKernelGGL(order_tiles, dim3(1), dim3(kOrderThreads), 0, stream, cost, order, n, n_items, split_per_cost,
                       max_split_log2, urgent_per_cost, graded, min_split_log2);
    return hipGetLastError();
}
#endif

template <typename R>
hipError_t launch_debug_shape(const ShapeRec<R>* shapes, int slot, int kind, uint32_t mode, uint32_t world_space,
                              const double* in, uint32_t n, double* out, hipStream_t stream) {
    (void)hipGetLastError();  // see launch_trace
    hipLaunchKernelGGL(debug_shape<R>, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, slot, kind, mode,
                       world_space, in, n, out);
    return hipGetLastError();
}
#if RTC_PRECISION != 2
template hipError_t launch_debug_shape<float>(const ShapeRec<float>*, int, int, uint32_t, uint32_t, const double*,
                                              uint32_t, double*, hipStream_t);
#endif
#if RTC_PRECISION != 1
template hipError_t launch_debug_shape<double>(const ShapeRec<double>*, int, int, uint32_t, uint32_t, const double*,
                                               uint32_t, double*, hipStream_t);
#endif

#if RTC_PRECISION != 2
hipError_t launch_canvas_signal(unsigned long long* flag, unsigned long long seq, hipStream_t stream) {
    (void)hipGetLastError();  // see launch_trace
    hipLaunchKernelGGL(canvas_signal, dim3(1), dim3(64), 0, stream, flag, seq);
    return hipGetLastError();
}
hipError_t launch_canvas_wait(const unsigned long long* flags, uint32_t n, unsigned long long seq,
                              unsigned long long timeout_ticks, int32_t* err, hipStream_t stream) {
    (void)hipGetLastError();  // see launch_trace
    hipLaunchKernelGGL(canvas_wait, dim3(1), dim3(64), 0, stream, flags, n, seq, timeout_ticks, err);
    return hipGetLastError();
}
#endif

#if RTC_PRECISION != 2
hipError_t launch_assemble(const void* gathered, void* image, uint32_t width, uint32_t height, uint32_t shards,
                           uint32_t strip_rows, uint32_t bpp, hipStream_t stream) {
    (void)hipGetLastError();  // see launch_trace
    const uint64_t row_bytes = (uint64_t)width * bpp;
    const bool wide = ((row_bytes | (uintptr_t)gathered | (uintptr_t)image) & 15) == 0;
    const uint64_t per_row = wide ? (row_bytes / 16 + 255) / 256 : 4;  // blocks per row (kernel's two paths)
    dim3 grid((uint32_t)std::min<uint64_t>(std::max<uint64_t>(per_row, 1), 64), height);
    hipLaunchKernelGGL(assemble_shards, grid, dim3(256), 0, stream, static_cast<const unsigned char*>(gathered),
                       static_cast<unsigned char*>(image), width, height, shards, strip_rows, bpp);
    return hipGetLastError();
}
#endif

#endif  // !RTC_VARIANT
#endif  // !RTC_JIT
#ifdef RTC_VARIANT
}  // namespace RTC_VARIANT
#endif
}  // namespace rtc
