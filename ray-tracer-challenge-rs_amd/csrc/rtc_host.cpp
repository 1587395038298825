// rtc_host.cpp — the C-ABI of include/rtc.h: context, world flattening and
// upload, launch of the gfx950 kernels, counters.
//
// Boundary it replaces: Camera::render / render_parallel
// (camera.rs:79-112) borrow `&World` and return an owned Canvas; here the
// caller hands the World as POD tables once (rt_scene_upload) and gets the
// canvas written into its own buffer per frame (rt_render / rt_render_device).
// There is no CPU fallback: without a HIP device every call that computes
// fails with RT_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rtc.h"
#include "flop_model.hpp"
#include "host_math.hpp"
#include "debug_knobs.hpp"
#include "rtc_context.hpp"
#include "rtc_internal.hpp"
#include "shape_identity.hpp"

namespace rtc {

template <typename R>
hipError_t launch_trace(const LaunchParams<R>& P, bool pool, bool dup, uint32_t grid, size_t dyn_lds,
                        hipStream_t stream);
template <typename R>
hipError_t occupancy(bool pool, bool lds, size_t dyn_lds, int* blocks_per_cu);

namespace sp {  // rtc_kernels_sp.o: the f32 pool kernel for worlds of spheres and planes only
template <typename R>
hipError_t launch_trace(const LaunchParams<R>& P, bool pool, bool dup, uint32_t grid, size_t dyn_lds,
                        hipStream_t stream);
}  // namespace sp
constexpr uint32_t kKindsSp = (1u << RT_SHAPE_SPHERE) | (1u << RT_SHAPE_PLANE);

hipError_t launch_order_tiles(uint32_t* cost, uint32_t* order, uint32_t n, uint32_t* n_items, float split_per_cost,
                              uint32_t max_split_log2, float urgent_per_cost, uint32_t graded, uint32_t min_split_log2,
                              hipStream_t stream);
template <typename R>
hipError_t launch_debug_shape(const ShapeRec<R>* shapes, int slot, int kind, uint32_t mode, uint32_t world_space,
                              const double* in, uint32_t n, double* out, hipStream_t stream);
hipError_t launch_assemble(const void* gathered, void* image, uint32_t width, uint32_t height, uint32_t shards,
                           uint32_t strip_rows, uint32_t bpp, hipStream_t stream);

namespace {
thread_local std::string g_error;
}

int set_error(int code, const std::string& msg) {
    g_error = msg;
    return code;
}


}  // namespace rtc

namespace rtc {
namespace {

// Copies run on the context's stream, never the null stream: HIP creates a
// hardware queue for the null stream at its first use, ~8 ms that a one-shot
// render would pay.  The caller synchronizes the stream before
// the host vector goes away.
template <typename T>
int upload(T** dst, const std::vector<T>& v, hipStream_t s) {
    if (v.empty()) {
        *dst = nullptr;
        return RT_OK;
    }
    RT_HIP(hipMalloc(reinterpret_cast<void**>(dst), v.size() * sizeof(T)));
    RT_HIP(hipMemcpyAsync(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return RT_OK;
}

}  // namespace

// World-space bounding sphere of a shape's intersection set, for the
// kernels' wave-level cull (wave_may_hit).  Acceleration only: a shape is
// skipped for a wave only when no lane's ray can meet this sphere at t >= 0,
// so it is padded well beyond the f32/f64 rounding of the local-space tests.
// Returns radius -1 for unbounded shapes (planes, open-ended cylinders,
// every cone) and for transforms whose forward matrix is not finite.
// Cones: a ray parallel to the side (|a| < EPSILON, |b| > EPSILON) gets the
// single root -c / 2b with no y-range test (cone.rs:97-99), anywhere on the
// infinite double cone, so no ball around the finite cone bounds a cone's
// entries (a random world's grazing ray found it: tests/test_gpu_random_worlds.py).
void bounding_sphere(const rt_shape_desc& d, double out[4]) {
    out[0] = out[1] = out[2] = 0.0;
    out[3] = -1.0;
    double c[3] = {0.0, 0.0, 0.0}, r = 0.0;
    const double lo = d.minimum, hi = d.maximum;
    switch (d.kind) {
        case RT_SHAPE_SPHERE: r = 1.0; break;
        case RT_SHAPE_CUBE: r = std::sqrt(3.0); break;
        case RT_SHAPE_CYLINDER: {
            if (!std::isfinite(lo) || !std::isfinite(hi) || !(lo <= hi)) return;
            const double half = 0.5 * (hi - lo);
            c[1] = 0.5 * (lo + hi);
            r = std::sqrt(1.0 + half * half);
            break;
        }
        case RT_SHAPE_TRIANGLE: {
            double p[3][3];
            for (int q = 0; q < 3; ++q) {
                p[0][q] = d.vertex_1[q];
                p[1][q] = d.vertex_1[q] + d.edge_1[q];
                p[2][q] = d.vertex_1[q] + d.edge_2[q];
            }
            for (int q = 0; q < 3; ++q) c[q] = (p[0][q] + p[1][q] + p[2][q]) / 3.0;
            for (auto& v : p)
                r = std::max(r, std::sqrt((v[0] - c[0]) * (v[0] - c[0]) + (v[1] - c[1]) * (v[1] - c[1]) +
                                          (v[2] - c[2]) * (v[2] - c[2])));
            break;
        }
        default: return;  // plane, cone
    }
    hm::M4 inv;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) inv.m[i][j] = d.inverse[4 * i + j];
    const hm::M4 f = hm::inverse(inv);
    // spectral norm of the linear part <= sqrt(max abs row sum of F^T F)
    double ftf[3][3] = {}, sigma2 = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) ftf[i][j] += f.m[k][i] * f.m[k][j];
    for (auto& row : ftf) sigma2 = std::max(sigma2, std::fabs(row[0]) + std::fabs(row[1]) + std::fabs(row[2]));
    double wc[3];
    for (int i = 0; i < 3; ++i) wc[i] = f.m[i][0] * c[0] + f.m[i][1] * c[1] + f.m[i][2] * c[2] + f.m[i][3];
    const double wr = r * std::sqrt(sigma2);
    const double scale = std::fabs(wc[0]) + std::fabs(wc[1]) + std::fabs(wc[2]) + wr;
    const double pad = 1e-3 * wr + 1e-4 * scale + 1e-4;
    if (!std::isfinite(wc[0]) || !std::isfinite(wc[1]) || !std::isfinite(wc[2]) || !std::isfinite(wr) ||
        wr + pad > 1e18)
        return;
    for (int i = 0; i < 3; ++i) out[i] = wc[i];
    out[3] = wr + pad;
}

// A sphere whose transformation is a similarity (rotation, uniform scale,
// translation): its world centre and radius^2, for the f32 kernels' roots in
// world space (rtc_internal.hpp kShapeSimilar, rtc_kernels.hip sphere_world).
// The linear part L of the forward transformation must satisfy
// L^T L = s^2 I to 1e-9 of s^2, far below the f32 rounding the kernels work
// at; shadow_puppets.yaml's backdrop (scaled 0.01 in z) keeps the
// object-space test.
bool similar_sphere(const rt_shape_desc& d, double centre[3], double* r2) {
    if (d.kind != RT_SHAPE_SPHERE) return false;
    hm::M4 inv;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) inv.m[i][j] = d.inverse[4 * i + j];
    if (inv.m[3][0] != 0.0 || inv.m[3][1] != 0.0 || inv.m[3][2] != 0.0 || inv.m[3][3] != 1.0) return false;
    const hm::M4 f = hm::inverse(inv);
    double g[3][3] = {};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) g[i][j] += f.m[k][i] * f.m[k][j];
    const double s2 = (g[0][0] + g[1][1] + g[2][2]) / 3.0;
    if (!(s2 > 0.0) || !std::isfinite(s2)) return false;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            if (!(std::fabs(g[i][j] - (i == j ? s2 : 0.0)) <= 1e-9 * s2)) return false;
    for (int i = 0; i < 3; ++i) {
        centre[i] = f.m[i][3];
        if (!std::isfinite(centre[i])) return false;
    }
    *r2 = s2;
    return true;
}

// A cube whose transformation has a diagonal linear part (rtc_internal.hpp
// kShapeAxisAligned): per axis the world coordinates of its object -1 and +1
// faces, the world |d| below which the axis counts as parallel (EPSILON over
// the axis's scale: the object direction is s d) and the scale's sign, for
// the f32 kernels' world-space slab test.  Off-diagonal terms within 1e-12 of
// the diagonal's size count as zero (far below f32 rounding).
bool axis_aligned_cube(const rt_shape_desc& d, double face_lo[3], double face_hi[3], double eps[3], double sgn[3]) {
    if (d.kind != RT_SHAPE_CUBE) return false;
    const double* m = d.inverse;  // rows of the inverse (row-major 4x4)
    if (m[12] != 0.0 || m[13] != 0.0 || m[14] != 0.0 || m[15] != 1.0) return false;
    double dmax = 0.0;
    for (int i = 0; i < 3; ++i) dmax = std::max(dmax, std::fabs(m[4 * i + i]));
    if (!(dmax > 0.0) || !std::isfinite(dmax)) return false;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            if (i != j && !(std::fabs(m[4 * i + j]) <= 1e-12 * dmax)) return false;
    for (int i = 0; i < 3; ++i) {
        const double sc = m[4 * i + i], t = m[4 * i + 3];
        if (sc == 0.0 || !std::isfinite(sc) || !std::isfinite(t)) return false;
        face_lo[i] = (-1.0 - t) / sc;
        face_hi[i] = (1.0 - t) / sc;
        eps[i] = 0.00000008 / std::fabs(sc);  // consts.rs EPSILON
        sgn[i] = sc > 0.0 ? 1.0 : -1.0;
    }
    return true;
}

// Device table order: by kind, then by identity class (the world index of
// the class's first shape), then by world index.  Without value-equal shapes
// this is world order within each kind.  The tie rule never depends on the
// table order (the kernels carry world indices), so the order only groups
// each class's members for the containers walk.
std::vector<uint32_t> table_order(const rt_shape_desc* shapes, uint32_t ns, const std::vector<uint32_t>& cls) {
    std::vector<uint32_t> order(ns);
    for (uint32_t i = 0; i < ns; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        if (shapes[a].kind != shapes[b].kind) return shapes[a].kind < shapes[b].kind;
        return cls[a] < cls[b];
    });
    return order;
}

template <typename R>
int build_world(rt_context* ctx, DeviceWorld<R>& w, const rt_shape_desc* shapes, uint32_t ns,
                const rt_material_desc* mats, uint32_t nm, const rt_pattern_desc* pats, uint32_t np,
                const rt_light_desc* lights, uint32_t nl, const std::vector<uint32_t>& cls) {
    w.release();
    std::vector<ShapeRec<R>> sh;
    std::vector<int32_t> begin(kNumKinds + 1, 0);
    const std::vector<uint32_t> order = table_order(shapes, ns, cls);
    size_t next = 0;
    for (int k = 0; k < kNumKinds; ++k) {
        begin[k] = (int32_t)sh.size();
        for (; next < order.size() && shapes[order[next]].kind == k; ++next) {
            const uint32_t i = order[next];
            const rt_shape_desc& d = shapes[i];
            ShapeRec<R> r{};
            for (int q = 0; q < 12; ++q) r.inv[q] = (R)d.inverse[q];
            double bs[4];
            bounding_sphere(d, bs);
            for (int q = 0; q < 3; ++q) r.bound[q] = (R)bs[q];
            // the device keeps r^2; unbounded is +inf for spheres and cubes
            // (their test has no branch), -1 for the other kinds (wave_may_hit)
            const bool branchless = d.kind == RT_SHAPE_SPHERE || d.kind == RT_SHAPE_CUBE;
            r.bound[3] = ctx->cull && bs[3] >= 0.0 ? (R)(bs[3] * bs[3])
                                                   : (branchless ? std::numeric_limits<R>::infinity() : (R)-1);
            r.ymin = (R)d.minimum;
            r.ymax = (R)d.maximum;
            for (int q = 0; q < 3; ++q) {
                r.tri[q] = (R)d.vertex_1[q];
                r.tri[3 + q] = (R)d.edge_1[q];
                r.tri[6 + q] = (R)d.edge_2[q];
                r.tri[9 + q] = (R)d.normal[q];
            }
            double centre[3], r2 = 0.0;
            const bool similar = similar_sphere(d, centre, &r2);
            if (similar) {
                for (int q = 0; q < 3; ++q) r.tri[q] = (R)centre[q];
                r.tri[3] = (R)r2;
            }
            double flo[3], fhi[3], feps[3], fsgn[3];
            const bool aligned = axis_aligned_cube(d, flo, fhi, feps, fsgn);
            if (aligned)
                for (int q = 0; q < 3; ++q) {
                    r.tri[q] = (R)flo[q];
                    r.tri[3 + q] = (R)fhi[q];
                    r.tri[6 + q] = (R)feps[q];
                    r.tri[9 + q] = (R)fsgn[q];
                }
            r.world_index = (int32_t)i;
            r.material = d.material;
            const bool class_end = next + 1 >= order.size() || cls[order[next + 1]] != cls[i];
            r.flags = (d.closed ? kShapeClosed : 0) | (class_end ? kShapeClassEnd : 0) | (similar ? kShapeSimilar : 0) | (aligned ? kShapeAxisAligned : 0) |
                      (int32_t)(cls[i] << kShapeClassShift);
            r.casts_shadow = mats[d.material].casts_shadow ? 1 : 0;
            sh.push_back(r);
        }
    }
    begin[kNumKinds] = (int32_t)sh.size();
    // world order -> (slot | kind << 24), padded to whole 16-byte words
    std::vector<int32_t> ws((sh.size() + 3) / 4 * 4, -1);
    for (int k = 0; k < kNumKinds; ++k)
        for (int32_t j = begin[k]; j < begin[k + 1]; ++j) ws[sh[j].world_index] = j | (k << 24);
    std::vector<MaterialRec<R>> mt(nm);
    bool any_secondary = false;
    for (uint32_t i = 0; i < nm; ++i) {
        const rt_material_desc& d = mats[i];
        MaterialRec<R>& m = mt[i];
        for (int q = 0; q < 3; ++q) m.color[q] = (R)d.color[q];
        m.ambient = (R)d.ambient;
        m.diffuse = (R)d.diffuse;
        m.specular = (R)d.specular;
        m.shininess = (R)d.shininess;
        m.reflectiveness = (R)d.reflectiveness;
        m.transparency = (R)d.transparency;
        m.refractive_index = (R)d.refractive_index;
        m.pattern = d.pattern;
        m.casts_shadow = d.casts_shadow;
        if (d.reflectiveness != 0.0 || d.transparency != 0.0) any_secondary = true;
    }
    std::vector<PatternRec<R>> pt(np);
    for (uint32_t i = 0; i < np; ++i) {
        const rt_pattern_desc& d = pats[i];
        PatternRec<R>& p = pt[i];
        for (int q = 0; q < 3; ++q) {
            p.color_a[q] = (R)d.color_a[q];
            p.color_b[q] = (R)d.color_b[q];
        }
        for (int q = 0; q < 12; ++q) p.inv[q] = (R)d.inverse[q];
        p.kind = d.kind;
        p.sub_a = d.sub_a;
        p.sub_b = d.sub_b;
    }
    std::vector<LightRec<R>> lt(nl);
    for (uint32_t i = 0; i < nl; ++i)
        for (int q = 0; q < 3; ++q) {
            lt[i].position[q] = (R)lights[i].position[q];
            lt[i].intensity[q] = (R)lights[i].intensity[q];
        }
    int rc;
    // shapes, materials, patterns and world_slot in one allocation, in the LDS layout
    const size_t image_bytes = world_lds_bytes<R>(sh.size(), nm, np);
    std::vector<unsigned char> img(image_bytes);
    size_t at = 0;
    auto put = [&](const void* src, size_t n) {
        if (n) std::memcpy(img.data() + at, src, n);
        at += n;
    };
    put(sh.data(), sh.size() * sizeof(ShapeRec<R>));
    put(mt.data(), mt.size() * sizeof(MaterialRec<R>));
    put(pt.data(), pt.size() * sizeof(PatternRec<R>));
    put(ws.data(), ws.size() * sizeof(int32_t));
    RT_HIP(hipMalloc(&w.image, std::max<size_t>(image_bytes, 16)));  // (an empty world still gets a buffer)
    if (image_bytes) RT_HIP(hipMemcpyAsync(w.image, img.data(), image_bytes, hipMemcpyHostToDevice, ctx->stream));
    w.carve(sh.size(), nm, np);
    if ((rc = upload(&w.lights, lt, ctx->stream))) {
        (void)hipStreamSynchronize(ctx->stream);  // the image copy may still read `img`
        return rc;
    }
    RT_HIP(hipStreamSynchronize(ctx->stream));  // (img and lt are host temporaries)
    if constexpr (sizeof(R) == 4) {  // the per-scene build's tables (capture_jit_table), from the host copies
        ctx->jit_shapes = sh;
        ctx->jit_lights = lt;
        ctx->jit_materials = mt;
        ctx->jit_pattern_recs = pt;
    }
    ctx->world_slot.assign(ws.begin(), ws.begin() + ns);
    w.scene.shapes = w.shapes;
    w.scene.materials = w.materials;
    w.scene.patterns = w.patterns;
    w.scene.lights = w.lights;
    w.scene.world_slot = w.world_slot;
    for (int k = 0; k <= kNumKinds; ++k) w.scene.kind_begin[k] = begin[k];
    w.scene.n_materials = (int32_t)nm;
    w.scene.n_patterns = (int32_t)np;
    w.scene.n_lights = (int32_t)nl;
    w.scene.any_secondary = any_secondary ? 1 : 0;
    return RT_OK;
}

int validate_scene(const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
                   const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights, uint32_t nl) {
    if ((ns && !shapes) || (nm && !mats) || (np && !pats) || (nl && !lights))
        return set_error(RT_ERR_INVALID, "rt_scene_upload: null table with nonzero count");
    for (uint32_t i = 0; i < ns; ++i) {
        if (shapes[i].kind < 0 || shapes[i].kind >= kNumKinds)
            return set_error(RT_ERR_INVALID, "shape " + std::to_string(i) + ": unknown kind");
        if (shapes[i].material < 0 || (uint32_t)shapes[i].material >= nm)
            return set_error(RT_ERR_INVALID, "shape " + std::to_string(i) + ": material index out of range");
    }
    for (uint32_t i = 0; i < nm; ++i)
        if (mats[i].pattern >= 0 && (uint32_t)mats[i].pattern >= np)
            return set_error(RT_ERR_INVALID, "material " + std::to_string(i) + ": pattern index out of range");
    for (uint32_t i = 0; i < np; ++i) {
        if (pats[i].kind < 0 || pats[i].kind > RT_PATTERN_TEST)
            return set_error(RT_ERR_INVALID, "pattern " + std::to_string(i) + ": unknown kind");
        if (pats[i].kind == RT_PATTERN_COMPLEX &&
            (pats[i].sub_a < 0 || pats[i].sub_b < 0 || (uint32_t)pats[i].sub_a >= np || (uint32_t)pats[i].sub_b >= np))
            return set_error(RT_ERR_INVALID, "pattern " + std::to_string(i) + ": bad sub-pattern index");
    }
    if (ns > 0xFFFFFF || nl > 0x7fffffff) return set_error(RT_ERR_INVALID, "table too large");
    return RT_OK;
}

uint32_t tile_rows_for(uint32_t height, uint32_t shards, uint32_t shard) {
    return shard_tile_rows(height, shards, shard);
}

// LIFO bound of a workgroup's ray pool (rays).  Block-lockstep generations
// pop at most `batch` rays from the top and push at most two children per
// ray, one level deeper, so the pool never holds more than
// kBlock + depth x batch.  A child past the bound would be dropped and
// flagged (RT_ERR_POOL), never written out of bounds.
uint32_t pool_capacity(uint32_t depth, uint32_t batch) {
    return (uint32_t)kBlock + depth * batch;
}

// Dynamic LDS of the pool (after the world tables): the item slots'
// accumulators, then `lcap` LIFO slots (a multiple of 8 keeps every array
// 16-byte aligned).
template <typename R>
size_t pool_lds_bytes(uint32_t lcap) {
    return (size_t)kTileSlots * 3 * kBlock * sizeof(PoolAcc<R>) + (size_t)lcap * (7 * sizeof(R) + sizeof(PoolMeta));
}

// Bound on any pixel of the pool kernel: a shaded hit adds at most
// bright_hit, its children carry at most bright_w of its weight.
double pixel_bound(double bright_hit, double bright_w, uint32_t depth) {
    double tree = 0.0, w = 1.0;
    for (uint32_t g = 0; g <= depth; ++g, w *= bright_w) tree += w;
    return bright_hit * tree;
}

// The pool kernel's fixed-point sums hold pixels up to 2^30 x 2^-acc_log2
// (f32: int32, acc_log2 >= kAccLog2Min) or 2^15 (f64: int64 multiples of
// 2^-48): a world that may exceed that (a TestPattern on an unbounded
// surface, or huge light intensities) is refused rather than wrapped.
int check_pixel_range(const rt_context* ctx, uint32_t depth, bool f32) {
    const double b = pixel_bound(ctx->bright_hit, ctx->bright_w, depth);
    const double lim = f32 ? std::ldexp(1.0, 30 - (int)kAccLog2Min) : std::ldexp(1.0, 14);
    if (!(b < lim))
        return set_error(RT_ERR_INVALID, "pixel colours of this world are unbounded for the ray pool's fixed-point sums "
                                         "(bound " + std::to_string(b) + " >= " + std::to_string(lim) +
                                         "; a TestPattern on an unbounded surface?)");
    return RT_OK;
}

// Scale of the f32 pool kernel's int32 pixel sums (rtc_internal.hpp
// PoolAcc): the largest 2^s with the world's brightest possible pixel below
// 2^30 / 2^s.  A shaded hit adds at most bright_hit (per light, the
// intensity times the material's colour x (ambient + diffuse) + specular,
// material.rs:83-114) and a hit's children carry at most bright_w of its
// weight (reflectiveness + transparency, world.rs:54-66: Schlick's R and
// 1 - R are in [0, 1]), so a pixel is below bright_hit x sum_{g<=depth} bright_w^g.
uint32_t acc_shift_f32(double bright_hit, double bright_w, uint32_t depth) {
    const double bound = std::max(pixel_bound(bright_hit, bright_w, depth), 1e-30);
    const int s = 30 - (int)std::ceil(std::log2(bound));
    return (uint32_t)std::min<int>(kAccLog2Max, std::max<int>(kAccLog2Min, s));
}

constexpr size_t kLdsPerCu = 160 * 1024;
// Static LDS of the tracer kernels (the pool kernel's per-wave LIFO tops and
// item tables and the counter flush: 400 B) plus headroom; the code-object
// metadata (tests/test_isa_budget.py) checks the real value.
constexpr size_t kStaticLds = 512;

struct LaunchShape {
    int per_cu;  // workgroups per CU the launch is planned for
    bool pool;
    uint32_t world_lds;  // world tables staged in LDS (bytes, 0 = none)
    uint32_t sched;
    uint32_t grid;
    size_t lds;
    uint32_t cap, lcap, batch;  // pool: LIFO bound, its LDS-resident part, pop batch
    uint32_t grid_tiles;        // the launch's tiles (the grid's upper bound)
};

// Cached occupancy (workgroups per CU) of one kernel instantiation at a
// given dynamic LDS size: the occupancy API's register/wave limit, and the
// LDS limit computed here from static + dynamic bytes (512-byte granules).
template <typename R>
int blocks_per_cu(rt_context* ctx, bool pool, bool lds_world, size_t lds, int* per_cu) {
    const int key = (pool ? 1 : 0) + (sizeof(R) == 8 ? 2 : 0) + (lds_world ? 4 : 0);
    if (ctx->occ_lds[key] == lds && ctx->occ_blocks[key] > 0) {
        *per_cu = ctx->occ_blocks[key];
        return RT_OK;
    }
    int api = 0;
    RT_HIP(occupancy<R>(pool, lds_world, lds, &api));
    const size_t per_block = (kStaticLds + lds + 511) / 512 * 512;
    const int by_lds = per_block ? (int)((size_t)kLdsPerCu / per_block) : api;
    *per_cu = std::min(api, by_lds);
    ctx->occ_lds[key] = lds;
    ctx->occ_blocks[key] = *per_cu;
    return RT_OK;
}

// LDS-resident part of the ray pool: as many slots as keep a pool kernel at
// the workgroups/CU its registers allow, `occ(lds, &blocks)` being its
// occupancy at a given dynamic LDS size; the rest of the bound spills to
// global memory.  *best: that workgroup count.
template <typename R, typename Occ>
int pool_lds_plan(rt_context* ctx, uint32_t world_lds, uint32_t cap, Occ&& occ, uint32_t* lcap, int* best_out) {
    constexpr uint32_t kMinRays = kBlock;
    int best = 0, rc;
    if ((rc = occ(world_lds + pool_lds_bytes<R>(kMinRays), &best))) return rc;
    if (best < 1) best = 1;
    const size_t rec = 7 * sizeof(R) + sizeof(PoolMeta);
    const size_t budget = (size_t)kLdsPerCu / (size_t)best;
    const size_t fixed = kStaticLds + world_lds + pool_lds_bytes<R>(0) + 511;
    uint32_t n = budget > fixed ? (uint32_t)((budget - fixed) / rec) : kMinRays;
    // one workgroup's LDS must also stay within the launch limit
    const size_t room = ctx->lds_per_block > fixed ? ctx->lds_per_block - fixed : 0;
    n = std::min<uint32_t>(n, (uint32_t)(room / rec));
    n = std::min<uint32_t>(cap, std::max<uint32_t>(kMinRays, n & ~7u));
    for (;;) {  // granule rounding: step down until `best` workgroups fit
        int got = 0;
        if ((rc = occ(world_lds + pool_lds_bytes<R>(n), &got))) return rc;
        if (got >= best || n <= kMinRays) break;
        n = std::max<uint32_t>(kMinRays, n - 8);
    }
    *lcap = n;
    if (best_out) *best_out = best;
    return RT_OK;
}

// ... for the static pool kernel (6 workgroups/CU for f32 at <= 80 VGPRs).
// RTC_DEBUG=pool_lds_rays=N overrides (A/B).
template <typename R>
int pool_lds_rays(rt_context* ctx, uint32_t world_lds, uint32_t cap, uint32_t* lcap) {
    if (ctx->pool_lds_rays > 0) {
        *lcap = std::min<uint32_t>(cap, std::max<uint32_t>(kBlock, ctx->pool_lds_rays & ~7u));
        return RT_OK;
    }
    const bool lw = world_lds != 0;
    return pool_lds_plan<R>(ctx, world_lds, cap,
                            [&](size_t lds, int* b) { return blocks_per_cu<R>(ctx, true, lw, lds, b); }, lcap, nullptr);
}

// LDS world of a per-scene kernel that takes the shape records from its
// instruction stream (rtc_kernels.hip kJitRecords: worlds of <= 255 shapes):
// the materials and patterns only.
template <typename R>
size_t jit_world_lds_bytes(const DevScene<R>& sc) {
    return (size_t)sc.n_materials * sizeof(MaterialRec<R>) + (size_t)sc.n_patterns * sizeof(PatternRec<R>);
}
#ifndef RTC_JIT_NO_RECORDS  // (A/B builds: -DRTC_JIT_NO_RECORDS keeps the whole world in LDS)
constexpr int32_t kJitRecordsMaxShapes = 255;
#else
constexpr int32_t kJitRecordsMaxShapes = -1;
#endif

// A per-scene pool kernel built for more waves/SIMD than the static one
// (rtc_jit.cpp jit_function): the pool's LDS share re-planned for the
// workgroups per CU its registers allow, as pool_lds_rays does for the
// static kernel, and the resident grid with it.
template <typename R>
int plan_pool_for(rt_context* ctx, hipFunction_t fn, LaunchShape& ls) {
    auto blocks = [&](size_t lds, int* per_cu) -> int {  // (blocks_per_cu's rule, for this function)
        int api = 0;
        RT_HIP(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&api, fn, kBlock, lds));
        const size_t per_block = (kStaticLds + lds + 511) / 512 * 512;
        *per_cu = std::min(api, (int)((size_t)kLdsPerCu / per_block));
        return RT_OK;
    };
    uint32_t n = 0;
    int best = 0, got = 0, rc;
    if ((rc = pool_lds_plan<R>(ctx, ls.world_lds, ls.cap, blocks, &n, &best))) return rc;
    if ((rc = blocks(ls.world_lds + pool_lds_bytes<R>(n), &got))) return rc;
    if (got <= ls.per_cu) return RT_OK;  // no more workgroups than planned: keep the plan
    ls.lcap = n;
    ls.lds = ls.world_lds + pool_lds_bytes<R>(n);
    ls.per_cu = got;
    const uint64_t resident = (uint64_t)got * (uint64_t)ctx->cu_count;
    ls.grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ls.grid_tiles, resident));
    return RT_OK;
}

template <typename R>
int plan_launch(rt_context* ctx, const DevScene<R>& sc, uint32_t depth, uint32_t n_tiles, LaunchShape& ls,
                bool jit_records = false) {
    ls.pool = sc.any_secondary && depth > 0;
    const size_t wb = jit_records ? std::max<size_t>(16, jit_world_lds_bytes(sc))
                                  : world_lds_bytes<R>(sc.kind_begin[kNumKinds], sc.n_materials, sc.n_patterns);
    // (a per-scene direct kernel takes its materials from constants too and
    // stages no world at all: rtc_kernels.hip kJitConstMaterials)
    ls.world_lds = (ctx->lds_world && wb <= kMaxWorldLds && !(jit_records && !ls.pool)) ? (uint32_t)wb : 0;
    ls.lds = ls.world_lds;
    ls.cap = ls.lcap = ls.batch = 0;
    ls.sched = ls.pool ? kSchedDynamic : ctx->sched_direct;
    int rc;
    if (ls.pool) {
        // (the pool kernel takes its items from the per-XCD queues only)
        ls.batch = kPoolBatch;
        ls.cap = pool_capacity(depth, ls.batch);
        if ((rc = pool_lds_rays<R>(ctx, ls.world_lds, ls.cap, &ls.lcap))) return rc;
        ls.lds += pool_lds_bytes<R>(ls.lcap);
    }
    int per_cu = 0;
    if ((rc = blocks_per_cu<R>(ctx, ls.pool, ls.world_lds != 0, ls.lds, &per_cu))) return rc;
    if (per_cu < 1) per_cu = 1;
    ls.per_cu = per_cu;
    const uint64_t resident = (uint64_t)per_cu * (uint64_t)ctx->cu_count;
    // The f32 direct kernel's static schedule runs 2.5x the resident grid: the
    // dispatcher starts the surplus workgroups as resident ones finish, which
    // evens out the last round.  Same-box sweep, three_sphere / shadow_puppets
    // 1080p (8160 tiles, 2048 resident at 8 waves/SIMD): 2048 34.4 / 42.0 us,
    // 3072 32.6 / 40.1, 4096 33.1 / 40.3, 5120 32.3 / 38.8, 6144 32.9 / 38.8,
    // 8160 (one tile each) 34.1 / 39.8; three_sphere 4K 115.6 -> 107.0 us.
    // The f64 kernel (3 waves/SIMD) measured 3.7% slower that way.
    const bool oversub = !ls.pool && ls.sched == kSchedStatic && sizeof(R) == 4;
    const uint64_t grid_cap = oversub ? std::max<uint64_t>(1, resident * ctx->direct_oversub10 / 10) : resident;
    ls.grid = ls.sched != kSchedGrid ? (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_tiles, grid_cap)) : n_tiles;
    ls.grid_tiles = n_tiles;
    return RT_OK;
}

// Same frame as the last pool launch?  (scene upload, canvas, shard, depth,
// precision, grid, camera; ray batches of rt_color_at are never
// cost-ordered)  Then hand its tiles out heaviest-first by the costs earlier
// launches recorded; every launch records its costs.  A frame's tile costs
// hardly change from one launch to the next, so the order is built
// (order_tiles) on launches 2 .. 1 + order_max_builds of a signature and then
// reused: order_tiles ran before every launch, 8 us per 1080p frame and 23 us
// per 4K frame of stream time ahead of the tracer.  A moved camera (the same
// frame otherwise) is ordered by the costs the previous camera's launch
// recorded: neighbouring frames of a camera path have similar tile costs.
// reflect_refract 1080p panning 0.1 degree per frame: 0.545 ms per frame in
// raster order, 0.528 reusing the first camera's order, 0.450 rebuilding
// from the previous frame's costs (scripts/camera_path.py), against 0.422
// for a repeated camera; metal, whose 0.1 ms frames gain little from any
// order, pays the 10 us sort (0.101 -> 0.107 ms).
template <typename R>
int plan_tile_order(rt_context* ctx, LaunchParams<R>& P, const rt_camera_desc* cam, uint32_t depth, uint32_t grid,
                    hipStream_t stream) {
    if (P.n_tiles > kItemTileMask + 1) return RT_OK;  // items carry 20 tile bits: raster order
    uint64_t h = 1469598103934665603ull;  // FNV-1a
    auto mix = [&h](const void* p, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    };
    const uint64_t fields[] = {ctx->scene_gen, P.n_tiles, P.width, P.height, P.shard_index, P.shard_count,
                               depth, sizeof(R), grid};
    mix(fields, sizeof(fields));
    const uint64_t geometry = h;
    if (cam) mix(cam, sizeof(*cam));
    if (ctx->order_capacity < P.n_tiles) {
        (void)hipFree(ctx->d_tile_cost);
        (void)hipFree(ctx->d_tile_order);
        ctx->d_tile_cost = ctx->d_tile_order = nullptr;
        ctx->order_capacity = 0;
        ctx->order_valid = ctx->order_built = false;
        RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_tile_cost), P.n_tiles * sizeof(uint32_t)));
        // (the kernel records a tile's cost as the maximum over its parts)
        RT_HIP(hipMemsetAsync(ctx->d_tile_cost, 0, P.n_tiles * sizeof(uint32_t), stream));
        // up to 2^kMaxSplitLog2 items per tile, then the item count
        RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_tile_order),
                         (((size_t)P.n_tiles << kMaxSplitLog2) + 1) * sizeof(uint32_t)));
        ctx->order_capacity = P.n_tiles;
    }
    const bool same = ctx->order_valid && ctx->order_sig == h;
    const bool moved = !same && ctx->order_valid && ctx->order_geometry == geometry;
    if (!same) ctx->order_builds = 0;
    if (!ctx->order_valid || ctx->order_geometry != geometry) ctx->order_built = false;
    uint32_t* n_items = ctx->d_tile_order + ((size_t)ctx->order_capacity << kMaxSplitLog2);
    if ((same || moved) && ctx->order_builds < kOrderBuilds) {
        const float split = ctx->split_factor > 0 ? (float)(ctx->split_factor / grid) : 0.0f;
        const float urgent = ctx->urgent_factor > 0 ? (float)(ctx->urgent_factor / grid) : 0.0f;
        RT_HIP(launch_order_tiles(ctx->d_tile_cost, ctx->d_tile_order, P.n_tiles, n_items, split, ctx->split_max,
                                  urgent, 1u, 0u, stream));
        ++ctx->order_builds;
        ctx->order_built = true;
    }
    if (ctx->order_built) {  // built from this frame's costs, or from the previous camera's frame
        P.tile_order = ctx->d_tile_order;
        P.item_count = n_items;
    } else if (P.shard_count == 1) {
        // No costs yet: tiles nearest the image centre first.  The order
        // depends on the canvas only, so it is built and uploaded once per
        // canvas size into its own buffer (order_tiles reuses d_tile_order).
        if (!ctx->d_cold_order || ctx->cold_w != P.width || ctx->cold_h != P.height) {
            const uint32_t n = P.n_tiles, tx = P.tiles_x;
            std::vector<std::pair<uint64_t, uint32_t>> key(n);
            const int64_t cx = (int64_t)P.width, cy = (int64_t)P.height;  // doubled centre
            for (uint32_t t = 0; t < n; ++t) {
                const int64_t x = 2 * (int64_t)((t % tx) * RT_TILE_W) + RT_TILE_W - cx;
                const int64_t y = 2 * (int64_t)((t / tx) * RT_TILE_H) + RT_TILE_H - cy;
                key[t] = {(uint64_t)(x * x + y * y), t};
            }
            std::sort(key.begin(), key.end());
            std::vector<uint32_t> v(n + 1);
            for (uint32_t i = 0; i < n; ++i) v[i] = key[i].second;
            v[n] = n;
            (void)hipFree(ctx->d_cold_order);
            ctx->d_cold_order = nullptr;
            RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_cold_order), v.size() * sizeof(uint32_t)));
            // (the launch's stream, not the null stream; v is a host temporary)
            RT_HIP(hipMemcpyAsync(ctx->d_cold_order, v.data(), v.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                  stream));
            RT_HIP(hipStreamSynchronize(stream));
            ctx->cold_w = P.width;
            ctx->cold_h = P.height;
        }
        P.tile_order = ctx->d_cold_order;
        P.item_count = ctx->d_cold_order + P.n_tiles;
    }
    P.tile_cost = ctx->d_tile_cost;
    ctx->order_sig = h;
    ctx->order_geometry = geometry;
    ctx->order_valid = true;
    return RT_OK;
}

int order_after_last(rt_context* ctx, hipStream_t stream) {
    if (ctx->launched && stream != ctx->last_stream) {
        RT_HIP(hipEventRecord(ctx->ev_order, ctx->last_stream));
        RT_HIP(hipStreamWaitEvent(stream, ctx->ev_order, 0));
    }
    ctx->last_stream = stream;
    ctx->launched = true;
    return RT_OK;
}

template <typename R>
int launch(rt_context* ctx, DeviceWorld<R>& w, const rt_camera_desc* cam, const double* d_rays, uint64_t n_rays,
           uint32_t depth, uint32_t out_format, uint32_t shard_index, uint32_t shard_count, void* out_device,
           hipStream_t stream, uint32_t flags = 0, bool image_rows = false) {
    int rc;
    LaunchParams<R> P{};
    P.image_rows = image_rows ? 1u : 0u;
    P.scene = w.scene;
    if (cam) {
        for (int q = 0; q < 12; ++q) P.cam.inv[q] = (R)cam->inverse[q];
        for (int q = 0; q < 3; ++q) P.cam.origin[q] = (R)cam->origin[q];
        P.cam.half_width = (R)cam->half_width;
        P.cam.half_height = (R)cam->half_height;
        P.cam.pixel_size = (R)cam->pixel_size;
        P.width = cam->width;
        P.height = cam->height;
        P.tiles_x = (cam->width + RT_TILE_W - 1) / RT_TILE_W;
        P.tile_rows = tile_rows_for(cam->height, shard_count, shard_index);
        P.n_tiles = P.tiles_x * P.tile_rows;
        P.tiles_x_magic = div_magic(P.tiles_x, P.n_tiles);
    } else {
        P.rays = d_rays;
        P.n_rays = n_rays;
        P.n_tiles = (uint32_t)((n_rays + kBlock - 1) / kBlock);
    }
    P.out = out_device;
    P.out_format = out_format;
    P.shard_index = shard_index;
    P.shard_count = shard_count;
    P.max_depth = depth;
    P.tile_counter = ctx->d_tile_counter;
    P.counters = ctx->d_counters;
    P.error_flag = ctx->d_error;
    if (flags & RT_FLAG_GENERATIONS) P.gen_counts = ctx->d_gen_counts;
    if (P.n_tiles == 0) return RT_OK;
    if ((rc = order_after_last(ctx, stream))) return rc;
    LaunchShape ls;
    rc = plan_launch<R>(ctx, w.scene, depth, P.n_tiles, ls);
    if (rc) return rc;
    // value-equal shapes (rt_scene_upload's identity classes) take the pool
    // kernel whose containers walk aggregates per class
    const bool dup = ctx->duplicate_shapes > 0;
    // large f32 frames run the per-scene build of the same kernel (rtc_jit.cpp);
    // a direct one takes the shape records and materials from its instruction
    // stream and is planned with no LDS world (pool builds keep the LDS world:
    // rtc_jit.cpp make_request)
    hipFunction_t jf = nullptr;
    if constexpr (sizeof(R) == 4) {
        // (the per-scene pool kernel keeps the stamps and item log: a stamped
        // launch times the kernel a warm renderer runs; the direct one has none)
        const uint32_t generic_only =
            RT_FLAG_NO_SHADE | RT_FLAG_NO_TRACE | RT_FLAG_GENERATIONS | (ls.pool ? 0u : RT_FLAG_STAMPS);
        const bool want = cam && !dup && !(flags & generic_only) &&
                          (ctx->jit_mode == RT_JIT_SYNC || (ctx->jit_mode >= RT_JIT_AUTO && P.n_tiles >= kJitMinTiles));
        if (want) {
            ++ctx->jit_frames;
            LaunchShape lj = ls;
            if (ctx->lds_world && !ls.pool && w.scene.kind_begin[kNumKinds] <= kJitRecordsMaxShapes &&
                (rc = plan_launch<R>(ctx, w.scene, depth, P.n_tiles, lj, true)))
                return rc;
            int waves = 0;
            if ((rc = jit_function(ctx, lj.pool, lj.world_lds != 0, lj.lds, lj.per_cu, &jf,
                                   (flags & RT_FLAG_NO_SKIPS) != 0, &waves)))
                return rc;
            if (jf && waves > 0 && (rc = plan_pool_for<R>(ctx, jf, lj))) return rc;
            if (jf) ls = lj;
        }
    }
    ctx->jit_used = jf != nullptr;
    P.pool_capacity = ls.cap;
    P.pool_lds_capacity = ls.lcap;
    P.pop_batch = ls.batch;
    if (ls.pool && (rc = check_pixel_range(ctx, depth, sizeof(R) == 4))) return rc;
    P.acc_log2 = acc_shift_f32(ctx->bright_hit, ctx->bright_w, depth);
    if (ls.cap > ls.lcap) {
        const size_t need = (size_t)ls.grid * 8 * (ls.cap - ls.lcap) * sizeof(R);
        if (ctx->spill_bytes < need) {
            (void)hipFree(ctx->d_spill);
            ctx->d_spill = nullptr;
            ctx->spill_bytes = 0;
            RT_HIP(hipMalloc(&ctx->d_spill, need));
            ctx->spill_bytes = need;
        }
        P.spill = ctx->d_spill;
        P.spill_blocks = (uint32_t)(ctx->spill_bytes / ((size_t)8 * (ls.cap - ls.lcap) * sizeof(R)));
    }
    P.persistent = ls.sched;
    P.flags = flags;
    P.world_lds = ls.world_lds;
    // Dynamic launches start from zeroed queue heads with no memset in
    // between: two sets alternate, both zeroed at context creation, and each
    // launch zeroes the other set for the next one (trace_pool; the
    // previous user of that set is complete by stream order).
    // The set flips only once the launch is enqueued: a launch that fails
    // before that leaves its set unused and still zero for the next one.
    // (pool launches only: the direct kernel reads no queue heads)
    const bool dynamic = ls.pool;
    if (dynamic) {
        const size_t set = (size_t)kTileQueues * kQueueStride;
        P.tile_counter = ctx->d_tile_counter + (ctx->head_set ? set : 0);
        P.next_tile_counter = ctx->d_tile_counter + (ctx->head_set ? 0 : set);
        if (ls.pool && ctx->tile_order && cam) {  // frames only: a ray batch's content is not in the signature
            if ((rc = plan_tile_order<R>(ctx, P, cam, depth, ls.grid, stream))) return rc;
        }
    }
    if (flags & RT_FLAG_STAMPS) {
        if (ctx->stamp_capacity < ls.grid) {
            (void)hipFree(ctx->d_stamps);
            ctx->d_stamps = nullptr;
            ctx->stamp_capacity = 0;
            RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_stamps), 2 * sizeof(unsigned long long) * ls.grid));
            ctx->stamp_capacity = ls.grid;
        }
        P.stamps = ctx->d_stamps;
        ctx->stamp_count = ls.grid;
        if (ls.pool) {  // every item of the launch: up to 2^kMaxSplitLog2 per tile
            const size_t items = (size_t)P.n_tiles << kMaxSplitLog2;
            if (ctx->item_log_capacity < items) {
                (void)hipFree(ctx->d_item_log);
                ctx->d_item_log = nullptr;
                ctx->item_log_capacity = 0;
                RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_item_log), (1 + 3 * items) * sizeof(uint64_t)));
                ctx->item_log_capacity = items;
            }
            RT_HIP(hipMemsetAsync(ctx->d_item_log, 0, sizeof(uint64_t), stream));
            P.item_log = ctx->d_item_log;
        }
    }
    // Worlds of spheres and planes only run the pool kernel built without the
    // other kinds' loops (rtc_kernels_sp.o; same pixels).  Same-box A/B:
    // reflect_refract -2.8%, refraction -6.7%.  The direct kernel measured
    // slower that way (three_sphere +2.5%), so it keeps every kind.  Both pool
    // builds are capped at the same waves/SIMD and use the same LDS, so the
    // occupancy planned above holds.  RTC_DEBUG=kind_variants=0 disables.
    uint32_t kinds = 0;
    for (int k = 0; k < kNumKinds; ++k)
        if (w.scene.kind_begin[k + 1] > w.scene.kind_begin[k]) kinds |= 1u << k;
    const bool sp = sizeof(R) == 4 && ls.pool && ctx->kind_variants && (kinds & ~kKindsSp) == 0 && !dup;
    if (flags & RT_FLAG_FAIL_LAUNCH) return set_error(RT_ERR_HIP, "launch refused (RT_FLAG_FAIL_LAUNCH)");
    if (jf) {
        const ShapeRec<R>* sh = P.scene.shapes;
        const MaterialRec<R>* mt = P.scene.materials;
        const PatternRec<R>* pt = P.scene.patterns;
        const LightRec<R>* lt = P.scene.lights;
        void* args[] = {&P, &sh, &mt, &pt, &lt};
        (void)hipGetLastError();
        RT_HIP(hipModuleLaunchKernel(jf, ls.grid, 1, 1, kBlock, 1, 1, (unsigned)ls.lds, stream, args, nullptr));
        if (dynamic) ctx->head_set ^= 1;
        return RT_OK;
    }
    if (hipError_t e = sp ? sp::launch_trace<R>(P, ls.pool, dup, ls.grid, ls.lds, stream)
                          : launch_trace<R>(P, ls.pool, dup, ls.grid, ls.lds, stream);
        e != hipSuccess)
        return set_error(RT_ERR_HIP, std::string("launch of the ") + (ls.pool ? "pool" : "direct") + " kernel (grid " +
                                         std::to_string(ls.grid) + ", dynamic LDS " + std::to_string(ls.lds) +
                                         " B, pool " + std::to_string(ls.lcap) + "/" + std::to_string(ls.cap) +
                                         " rays in LDS): " + hipGetErrorString(e));
    if (dynamic) ctx->head_set ^= 1;
    return RT_OK;
}

InitTrace::InitTrace(const char* what) : what_(what), on_(debug_knob("trace_init", nullptr)) {
    t0_ = t_ = std::chrono::steady_clock::now();
}
void InitTrace::step(const char* name) {
    if (!on_) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[rtc init] %s: %s %.3f ms (%.3f ms total)\n", what_, name,
                 std::chrono::duration<double, std::milli>(now - t_).count(),
                 std::chrono::duration<double, std::milli>(now - t0_).count());
    t_ = now;
}

int check_ready(rt_context* ctx) {
    if (!ctx) return set_error(RT_ERR_INVALID, "null context");
    if (!ctx->have_scene) return set_error(RT_ERR_NO_SCENE, "render before rt_scene_upload");
    return RT_OK;
}

int check_options(const rt_render_options* o) {
    if (!o) return set_error(RT_ERR_INVALID, "null options");
    if (o->precision > RT_PRECISION_F64) return set_error(RT_ERR_INVALID, "unknown precision");
    if (o->out_format > RT_OUT_U8) return set_error(RT_ERR_INVALID, "unknown output format");
    if (o->max_depth > RT_MAX_SUPPORTED_DEPTH) return set_error(RT_ERR_INVALID, "max_depth above RT_MAX_SUPPORTED_DEPTH");
    if (o->shard_count == 0 || o->shard_index >= o->shard_count) return set_error(RT_ERR_INVALID, "bad shard");
    return RT_OK;
}

int ensure_scratch(rt_context* ctx, size_t bytes) {
    if (ctx->scratch_bytes >= bytes) return RT_OK;
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    ctx->d_scratch = nullptr;
    ctx->scratch_bytes = 0;
    RT_HIP(hipMalloc(&ctx->d_scratch, bytes));
    ctx->scratch_bytes = bytes;
    return RT_OK;
}

int read_counters(rt_context* ctx, unsigned long long out[kNumCounters]) {
    std::vector<unsigned long long> shards((size_t)kCounterShards * kNumCounters);
    RT_HIP(hipMemcpy(shards.data(), ctx->d_counters, shards.size() * sizeof(unsigned long long),
                     hipMemcpyDeviceToHost));
    for (int i = 0; i < kNumCounters; ++i) out[i] = 0;
    for (int s = 0; s < kCounterShards; ++s)
        for (int i = 0; i < kNumCounters; ++i) out[i] += shards[(size_t)s * kNumCounters + i];
    return RT_OK;
}

void fill_stats(rt_context* ctx, const unsigned long long before[kNumCounters],
                const unsigned long long after[kNumCounters], float ms, rt_stats* s) {
    uint64_t d[kNumCounters];
    for (int i = 0; i < kNumCounters; ++i) d[i] = after[i] - before[i];
    s->primary = d[0];
    s->shadow = d[1];
    s->reflect = d[2];
    s->refract = d[3];
    s->shaded = d[4];
    s->lit_patterned = d[5];
    s->refract_evals = d[6];
    s->schlick_evals = d[7];
    s->kernel_ms = ms;
    s->algorithmic_flops = algorithmic_flops(ctx->flops, *s);
    s->gather_ms = 0.0;
    s->frame_ms = ms;
    s->n_shards = 1;
    s->reserved = 0;
}

int ensure_host_counters(rt_context* ctx) {
    if (ctx->h_counters) return RT_OK;
    const size_t cbytes = 2 * (size_t)kCounterShards * kNumCounters * sizeof(unsigned long long) + 64;
    RT_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_counters), cbytes, hipHostMallocDefault));
    return RT_OK;
}

// Device scratch -> the caller's host buffer, enqueued on ctx->stream after
// the render.  A pageable hipMemcpyAsync runs at the PCIe rate here (the
// runtime pipelines its own pinned staging): measured on MI355X for a 1080p
// f32 frame (24.9 MB) into a canvas kept across frames, 0.52 ms per whole
// rt_render call; a pinned staging buffer copied out by 4 host threads as
// each of 8 DMA chunks landed took 0.71 ms (scripts/host_frame_probe.py).
// A canvas allocated per call pays its page faults on top (~0.3 ms at 1080p).
int copy_to_host(rt_context* ctx, void* out, size_t bytes) {
    RT_HIP(hipMemcpyAsync(out, ctx->d_scratch, bytes, hipMemcpyDeviceToHost, ctx->stream));
    return RT_OK;
}

int check_pool_error(rt_context* ctx) {
    int32_t err = 0;
    RT_HIP(hipMemcpyAsync(&err, ctx->d_error, sizeof(err), hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    if (err) {
        RT_HIP(hipMemsetAsync(ctx->d_error, 0, sizeof(int32_t), ctx->stream));
        return set_error(RT_ERR_POOL, device_error_text(err));
    }
    return RT_OK;
}

}  // namespace rtc

using namespace rtc;

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

const char* rt_last_error(void) { return rtc::g_error.c_str(); }

int rt_device_count(int* count) {
    if (!count) return set_error(RT_ERR_INVALID, "null count");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return RT_OK;
}

int rt_context_create(int device_ordinal, rt_context** out) { return create_device_context(device_ordinal, out); }

int rt_context_destroy(rt_context* ctx) {
    if (!ctx) return RT_OK;
    for (rt_context* p : ctx->peers) destroy_device_context(p);
    ctx->peers.clear();
    destroy_device_context(ctx);
    return RT_OK;
}

}  // extern "C"

namespace rtc {

int create_device_context(int device_ordinal, rt_context** out) {
    if (!out) return set_error(RT_ERR_INVALID, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return set_error(RT_ERR_NO_DEVICE, "no HIP device available (the render path has no CPU fallback)");
    if (device_ordinal < 0 || device_ordinal >= n) return set_error(RT_ERR_INVALID, "device ordinal out of range");
    // RTC_DEBUG=trace_init=1: milliseconds of each step of context creation on
    // stderr (the one-shot render's breakdown)
    InitTrace tr("context");
    auto ctx = std::make_unique<rt_context>();
    ctx->device = device_ordinal;
    RT_HIP(hipSetDevice(device_ordinal));
    tr.step("hipSetDevice");
    // two attributes instead of hipGetDeviceProperties (which fills every
    // field of the struct); the gfx target for the per-scene builds is read
    // when the first build needs it (device_arch, rtc_jit.cpp)
    int cus = 0, lds = 0;
    RT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_ordinal));
    RT_HIP(hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device_ordinal));
    tr.step("hipDeviceGetAttribute x2");
    ctx->cu_count = cus;
    ctx->lds_per_block = (size_t)lds;  // launch limit of static + dynamic LDS
    // A/B and diagnostic switches (debug_knobs.hpp: RTC_DEBUG=key=value,...)
    std::string v;
    // direct-kernel tile scheduling: "grid" (one workgroup per tile, the
    // hardware dispatcher balances) or "static" (resident grid, fixed stride)
    if (debug_knob("sched_direct", &v)) {
        if (v == "grid") ctx->sched_direct = kSchedGrid;
        else if (v == "static") ctx->sched_direct = kSchedStatic;
    }
    if (debug_knob("lds_world", &v)) ctx->lds_world = v != "0";
    if (debug_knob("cull", &v)) ctx->cull = v != "0";
    if (debug_knob("kind_variants", &v)) ctx->kind_variants = v != "0";
    if (debug_knob("pool_lds_rays", &v)) ctx->pool_lds_rays = (uint32_t)std::atoi(v.c_str());
    if (debug_knob("tile_order", &v)) ctx->tile_order = v != "0";
    if (debug_knob("split", &v)) ctx->split_factor = std::atof(v.c_str());
    if (debug_knob("split_max", &v))
        ctx->split_max = (uint32_t)std::min<int>((int)kMaxSplitLog2, std::max(0, std::atoi(v.c_str())));
    if (debug_knob("urgent", &v)) ctx->urgent_factor = std::atof(v.c_str());
    if (debug_knob("direct_oversub", &v)) ctx->direct_oversub10 = (uint32_t)std::max(1, std::atoi(v.c_str()));
    // RTC_JIT: the per-scene build mode (rt_context_set_jit's values), a user setting
    if (const char* e = std::getenv("RTC_JIT"))
        ctx->jit_mode = (e[0] >= '0' && e[0] <= '3' && !e[1]) ? e[0] - '0' : RT_JIT_AUTO;
    RT_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    tr.step("hipStreamCreate");
    RT_HIP(hipEventCreate(&ctx->ev_start));
    RT_HIP(hipEventCreate(&ctx->ev_stop));
    RT_HIP(hipEventCreateWithFlags(&ctx->ev_order, hipEventDisableTiming));
    tr.step("hipEventCreate x3");
    const size_t qbytes = 2 * (size_t)kTileQueues * kQueueStride * sizeof(unsigned long long);  // two sets
    RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_tile_counter), qbytes));
    tr.step("hipMalloc");
    // (on the context's stream: the null stream's queue would cost ~8 ms more)
    RT_HIP(hipMemsetAsync(ctx->d_tile_counter, 0, qbytes, ctx->stream));
    tr.step("hipMemsetAsync (first)");
    const size_t counter_bytes = (size_t)kCounterShards * kNumCounters * sizeof(unsigned long long);
    RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_counters), counter_bytes));
    RT_HIP(hipMemsetAsync(ctx->d_counters, 0, counter_bytes, ctx->stream));
    RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_error), sizeof(int32_t)));
    RT_HIP(hipMemsetAsync(ctx->d_error, 0, sizeof(int32_t), ctx->stream));
    const size_t gen_bytes = 2 * (size_t)kGenSlots * sizeof(unsigned long long);
    RT_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_gen_counts), gen_bytes));
    RT_HIP(hipMemsetAsync(ctx->d_gen_counts, 0, gen_bytes, ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    tr.step("hipMalloc+hipMemsetAsync x3, sync");
    *out = ctx.release();
    return RT_OK;
}

void destroy_device_context(rt_context* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();  // launches on caller streams too
    for (auto& c : ctx->canvases) {
        if (c.second.owned) (void)hipFree(c.first);
        else (void)hipIpcCloseMemHandle(c.first);
    }
    ctx->canvases.clear();
    ctx->w32.release();
    ctx->w64.release();
    (void)hipFree(ctx->d_tile_counter);
    (void)hipFree(ctx->d_counters);
    (void)hipFree(ctx->d_error);
    (void)hipFree(ctx->d_gen_counts);
    (void)hipFree(ctx->d_scratch);
    (void)hipFree(ctx->d_stamps);
    (void)hipFree(ctx->d_item_log);
    (void)hipFree(ctx->d_spill);
    (void)hipFree(ctx->d_tile_cost);
    (void)hipFree(ctx->d_tile_order);
    (void)hipFree(ctx->d_cold_order);
    if (ctx->ev_start) (void)hipEventDestroy(ctx->ev_start);
    if (ctx->ev_stop) (void)hipEventDestroy(ctx->ev_stop);
    if (ctx->ev_order) (void)hipEventDestroy(ctx->ev_order);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    (void)hipFree(ctx->d_strip);
    (void)hipFree(ctx->d_gathered);
    (void)hipFree(ctx->d_status);
    if (ctx->h_counters) (void)hipHostFree(ctx->h_counters);
    for (hipEvent_t e : {ctx->ev_render0, ctx->ev_render1, ctx->ev_gather1})
        if (e) (void)hipEventDestroy(e);
    delete ctx;
}

}  // namespace rtc

extern "C" {

int rt_scene_upload(rt_context* ctx, const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats,
                    uint32_t nm, const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights,
                    uint32_t nl) {
    if (!ctx) return set_error(RT_ERR_INVALID, "null context");
    if (ctx->comm) return group_scene_upload(ctx, shapes, ns, mats, nm, pats, np, lights, nl);
    int rc = validate_scene(shapes, ns, mats, nm, pats, np, lights, nl);
    if (rc) return rc;
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(hipDeviceSynchronize());  // launches on caller streams may still read the old tables
    return build_scene(ctx, shapes, ns, mats, nm, pats, np, lights, nl);
}

}  // extern "C"

namespace rtc {

// Largest |coordinate| of a point of the shape's surface in object space
// (+inf for an unbounded surface): the reach of a TestPattern on it.
double object_extent(const rt_shape_desc& d) {
    const double inf = std::numeric_limits<double>::infinity();
    switch (d.kind) {
        case RT_SHAPE_SPHERE:
        case RT_SHAPE_CUBE: return 1.0;
        case RT_SHAPE_CYLINDER:
            return std::isfinite(d.minimum) && std::isfinite(d.maximum)
                       ? std::max({1.0, std::fabs(d.minimum), std::fabs(d.maximum)})
                       : inf;
        case RT_SHAPE_CONE:
            return std::isfinite(d.minimum) && std::isfinite(d.maximum)
                       ? std::max(std::fabs(d.minimum), std::fabs(d.maximum))
                       : inf;
        case RT_SHAPE_TRIANGLE: {
            double e = 0.0;
            for (int k = 0; k < 3; ++k)
                e = std::max({e, std::fabs(d.vertex_1[k]), std::fabs(d.vertex_1[k] + d.edge_1[k]),
                              std::fabs(d.vertex_1[k] + d.edge_2[k])});
            return e;
        }
        default: return inf;  // plane
    }
}

// The brightness bound of acc_shift_f32 for these tables: the largest
// colour a material can show (its colour, the colours of every pattern its
// pattern reaches, and for a TestPattern, pattern.rs:55-58, the pattern-space
// point itself: bounded by the surface's object-space extent through the
// material's pattern transform, +inf on an unbounded surface), times the
// lights' intensities and the Phong coefficients.
void scene_brightness(const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
                      const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights, uint32_t nl,
                      double* bright_hit, double* bright_w) {
    // per material: the colours its pattern chain may return, and whether a
    // TestPattern is among them
    std::vector<double> col(nm, 0.0);
    std::vector<char> test(nm, 0);
    for (uint32_t i = 0; i < nm; ++i) {
        for (int c = 0; c < 3; ++c) col[i] = std::max(col[i], std::fabs(mats[i].color[c]));
        std::vector<int32_t> todo;
        std::vector<char> seen(np, 0);
        if (mats[i].pattern >= 0 && (uint32_t)mats[i].pattern < np) todo.push_back(mats[i].pattern);
        while (!todo.empty()) {
            const int32_t q = todo.back();
            todo.pop_back();
            if (q < 0 || (uint32_t)q >= np || seen[q]) continue;
            seen[q] = 1;
            const rt_pattern_desc& pd = pats[q];
            if (pd.kind == RT_PATTERN_TEST) test[i] = 1;
            else if (pd.kind == RT_PATTERN_COMPLEX) todo.insert(todo.end(), {pd.sub_a, pd.sub_b});
            else
                for (int c = 0; c < 3; ++c) col[i] = std::max({col[i], std::fabs(pd.color_a[c]), std::fabs(pd.color_b[c])});
        }
    }
    for (uint32_t s = 0; s < ns; ++s) {  // a TestPattern's colour: the pattern-space point
        const int32_t m = shapes[s].material;
        if (m < 0 || (uint32_t)m >= nm || !test[m]) continue;
        const double ext = object_extent(shapes[s]) * (1.0 + 1e-3) + 1e-3;  // (over_point: a hair off the surface)
        const double* inv = pats[mats[m].pattern].inverse;  // (a complex pattern's subs use its transform)
        for (int r = 0; r < 3; ++r) {
            const double v = (std::fabs(inv[4 * r]) + std::fabs(inv[4 * r + 1]) + std::fabs(inv[4 * r + 2])) * ext +
                             std::fabs(inv[4 * r + 3]);
            col[m] = std::max(col[m], std::isnan(v) ? std::numeric_limits<double>::infinity() : v);
        }
    }
    // Children's weight: a reflective and transparent material mixes them as
    // r·R + t·(1 − R) (world.rs:59-63), at most max(r, t) while Schlick's R
    // stays in [0, 1] -- true when every refractive index is positive (r0 of
    // computed_hit.rs:62 in [0, 1), cos in [0, 1]; TIR gives R = 1); the
    // margin covers cos a rounding past 1 on an unrenormalised refracted
    // direction (world.rs:150).  Otherwise the children add: |r| + |t|.
    bool ri_positive = true;
    for (uint32_t i = 0; i < nm; ++i) ri_positive = ri_positive && mats[i].refractive_index > 0.0;
    double per_light = 0.0, w = 0.0;
    for (uint32_t i = 0; i < nm; ++i) {
        const rt_material_desc& m = mats[i];
        per_light = std::max(per_light, col[i] * (std::fabs(m.ambient) + std::fabs(m.diffuse)) + std::fabs(m.specular));
        const bool mixed = ri_positive && m.reflectiveness > 0.0 && m.transparency > 0.0;
        w = std::max(w, mixed ? std::max(m.reflectiveness, m.transparency) * (1.0 + 1e-6)
                              : std::fabs(m.reflectiveness) + std::fabs(m.transparency));
    }
    double hit = 0.0;
    for (uint32_t l = 0; l < nl; ++l) {
        double in = 0.0;
        for (int k = 0; k < 3; ++k) in = std::max(in, std::fabs(lights[l].intensity[k]));
        hit += in * per_light;
    }
    *bright_hit = std::isfinite(hit) ? hit : std::numeric_limits<double>::infinity();
    *bright_w = std::isfinite(w) ? w : std::numeric_limits<double>::infinity();
}

int build_scene(rt_context* ctx, const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
                const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights, uint32_t nl) {
    int rc;
    ctx->have_scene = false;
    std::vector<uint32_t> cls;  // value-identity classes (shape_identity.hpp)
    ctx->duplicate_shapes = ident::shape_classes(shapes, ns, mats, pats, cls);
    if ((rc = build_world<float>(ctx, ctx->w32, shapes, ns, mats, nm, pats, np, lights, nl, cls))) return rc;
    if ((rc = capture_jit_table(ctx))) return rc;
    if ((rc = build_world<double>(ctx, ctx->w64, shapes, ns, mats, nm, pats, np, lights, nl, cls))) return rc;
    ctx->flops = FlopScene{};
    for (uint32_t i = 0; i < ns; ++i) {
        const rt_shape_desc& d = shapes[i];
        ctx->flops.per_ray += shape_test_flops(d.kind, d.closed != 0);
    }
    ctx->flops.n_lights = nl;
    scene_brightness(shapes, ns, mats, nm, pats, np, lights, nl, &ctx->bright_hit, &ctx->bright_w);
    ctx->have_scene = true;
    ++ctx->scene_gen;  // invalidates the recorded tile costs
    return RT_OK;
}

int fetch_jit_tables(rt_context* ctx) {
    const DevScene<float>& sc = ctx->w32.scene;
    ctx->jit_shapes.assign(sc.kind_begin[kNumKinds], ShapeRec<float>{});
    ctx->jit_lights.assign(sc.n_lights, LightRec<float>{});
    ctx->jit_materials.assign(sc.n_materials, MaterialRec<float>{});
    ctx->jit_pattern_recs.assign(sc.n_patterns, PatternRec<float>{});
    auto get = [&](auto& v, const void* src) -> hipError_t {
        return v.empty() ? hipSuccess
                         : hipMemcpyAsync(v.data(), src, v.size() * sizeof(v[0]), hipMemcpyDeviceToHost, ctx->stream);
    };
    RT_HIP(get(ctx->jit_shapes, ctx->w32.shapes));
    RT_HIP(get(ctx->jit_lights, ctx->w32.lights));
    RT_HIP(get(ctx->jit_materials, ctx->w32.materials));
    RT_HIP(get(ctx->jit_pattern_recs, ctx->w32.patterns));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int capture_jit_table(rt_context* ctx) {
    // (jit_shapes, jit_lights, jit_materials, jit_pattern_recs: build_world<float>'s host tables)
    for (int k = 0; k <= kNumKinds; ++k) ctx->jit_begin[k] = ctx->w32.scene.kind_begin[k];
    const std::vector<MaterialRec<float>>& mats = ctx->jit_materials;
    ctx->jit_patterns = std::any_of(mats.begin(), mats.end(), [](const MaterialRec<float>& m) { return m.pattern >= 0; });
    ctx->jit_transparent =
        std::any_of(mats.begin(), mats.end(), [](const MaterialRec<float>& m) { return m.transparency != 0.0f; });
    ctx->jit_pattern_kinds = 0;
    for (const PatternRec<float>& q : ctx->jit_pattern_recs)  // every kind a pattern_color walk can meet (complex sub-patterns included)
        ctx->jit_pattern_kinds |= 1u << std::min<uint32_t>((uint32_t)q.kind, RT_PATTERN_TEST);
    for (int v = 0; v < rt_context::kJitVariants; ++v) {
        ctx->jit_fn[v] = nullptr;
        ctx->jit_build[v].reset();
        ctx->jit_rejected[v] = ctx->jit_owner[v] = false;
    }
    ctx->jit_frames = 0;
    ctx->jit_failed = false;
    ctx->jit_log.clear();
    return RT_OK;
}

int launch_frame(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, uint32_t shard_index,
                 uint32_t shard_count, void* out_device, hipStream_t s, bool image_rows) {
    RT_HIP(hipSetDevice(ctx->device));
    if (o->precision == RT_PRECISION_F32)
        return launch<float>(ctx, ctx->w32, cam, nullptr, 0, o->max_depth, o->out_format, shard_index, shard_count,
                             out_device, s, o->flags, image_rows);
    return launch<double>(ctx, ctx->w64, cam, nullptr, 0, o->max_depth, o->out_format, shard_index, shard_count,
                          out_device, s, o->flags, image_rows);
}

// ------------------------------------------------------------ peer canvas
unsigned long long* canvas_flags(void* canvas, uint64_t image_bytes) {
    return reinterpret_cast<unsigned long long*>(static_cast<unsigned char*>(canvas) + canvas_flag_offset(image_bytes));
}

unsigned long long timeout_ticks(double timeout_ms) {  // s_memrealtime runs at 100 MHz
    return timeout_ms < 0 ? ~0ull : (unsigned long long)(timeout_ms * 1e5);
}

// After a canvas's flags (n_flags ready flags + the release flag): a trailer
// {image bytes, n_flags}, so rt_canvas_open can check the caller's sizes
// against the creator's instead of placing its flags at a wrong offset.
size_t canvas_flag_bytes(uint32_t n_flags) { return ((size_t)n_flags + 1 + 2) * sizeof(unsigned long long); }

// The canvas is fine-grained device memory: other GPUs store pixels and
// flags into it over xGMI while the owner's canvas_wait polls the flags, and
// the owner then copies the image out.  In coarse-grained memory the owner's
// L2 may keep a line (a flag it polled, pixels it copied out last frame) that
// a peer's store to HBM never updates, and a system-scope acquire does not
// invalidate such lines; fine-grained lines are the ones its acquire
// (canvas_wait) invalidates and its kernels' releases write back.
int canvas_create(rt_context* ctx, uint64_t bytes, uint32_t n_flags, void** canvas) {
    RT_HIP(hipSetDevice(ctx->device));
    const size_t flag_bytes = canvas_flag_bytes(n_flags);
    void* p = nullptr;
    RT_HIP(hipExtMallocWithFlags(&p, canvas_flag_offset(bytes) + flag_bytes, hipDeviceMallocFinegrained));
    std::vector<unsigned long long> tail((size_t)n_flags + 3, 0ull);
    tail[n_flags + 1] = bytes;
    tail[n_flags + 2] = n_flags;
    if (hipError_t e = hipMemcpy(canvas_flags(p, bytes), tail.data(), flag_bytes, hipMemcpyHostToDevice);
        e != hipSuccess) {
        (void)hipFree(p);
        return set_error(RT_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
    }
    ctx->canvases[p] = {bytes, n_flags, true};
    *canvas = p;
    return RT_OK;
}

int canvas_close(rt_context* ctx, void* canvas) {
    auto it = ctx->canvases.find(canvas);
    if (it == ctx->canvases.end()) return set_error(RT_ERR_INVALID, "not a canvas of this context");
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(hipDeviceSynchronize());
    const bool owned = it->second.owned;
    ctx->canvases.erase(it);
    if (owned) RT_HIP(hipFree(canvas));
    else RT_HIP(hipIpcCloseMemHandle(canvas));
    return RT_OK;
}

}  // namespace rtc

extern "C" {

int rt_canvas_create(rt_context* ctx, uint64_t bytes, uint32_t n_flags, void** canvas,
                     uint8_t handle[RT_IPC_HANDLE_BYTES]) {
    static_assert(sizeof(hipIpcMemHandle_t) == RT_IPC_HANDLE_BYTES, "RT_IPC_HANDLE_BYTES must match hipIpcMemHandle_t");
    if (!ctx || !canvas || n_flags == 0 || bytes == 0) return set_error(RT_ERR_INVALID, "rt_canvas_create: bad arguments");
    int rc = canvas_create(ctx, bytes, n_flags, canvas);
    if (rc || !handle) return rc;
    hipIpcMemHandle_t h;
    if (hipError_t e = hipIpcGetMemHandle(&h, *canvas); e != hipSuccess) {
        (void)canvas_close(ctx, *canvas);
        *canvas = nullptr;
        return set_error(RT_ERR_HIP, std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e));
    }
    std::memcpy(handle, &h, sizeof h);
    return RT_OK;
}

int rt_canvas_open(rt_context* ctx, const uint8_t handle[RT_IPC_HANDLE_BYTES], uint64_t bytes, uint32_t n_flags,
                   void** canvas) {
    if (!ctx || !handle || !canvas || n_flags == 0 || bytes == 0)
        return set_error(RT_ERR_INVALID, "rt_canvas_open: bad arguments");
    RT_HIP(hipSetDevice(ctx->device));
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof h);
    void* p = nullptr;
    RT_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    // the creator's sizes, from the canvas's trailer (inside the mapped range only)
    hipDeviceptr_t base = nullptr;
    size_t range = 0;
    const size_t need = canvas_flag_offset(bytes) + canvas_flag_bytes(n_flags);
    unsigned long long tail[2] = {0, 0};
    const bool fits = hipMemGetAddressRange(&base, &range, (hipDeviceptr_t)p) == hipSuccess &&
                      static_cast<char*>(p) + need <= static_cast<char*>(base) + range;
    if (!fits || hipMemcpy(tail, canvas_flags(p, bytes) + n_flags + 1, sizeof tail, hipMemcpyDeviceToHost) != hipSuccess ||
        tail[0] != bytes || tail[1] != n_flags) {
        (void)hipIpcCloseMemHandle(p);
        return set_error(RT_ERR_INVALID, "rt_canvas_open: bytes / n_flags differ from the creator's (" +
                                             std::to_string(tail[0]) + " / " + std::to_string(tail[1]) + ")");
    }
    ctx->canvases[p] = {bytes, n_flags, false};
    *canvas = p;
    return RT_OK;
}

int rt_canvas_close(rt_context* ctx, void* canvas) {
    if (!ctx || !canvas) return set_error(RT_ERR_INVALID, "rt_canvas_close: bad arguments");
    return canvas_close(ctx, canvas);
}

int rt_render_to_canvas(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* canvas,
                        uint64_t seq, double timeout_ms, void* hip_stream) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if ((rc = check_options(o))) return rc;
    if (ctx->comm) return set_error(RT_ERR_INVALID, "rt_render_to_canvas takes a single-GPU context");
    auto it = ctx->canvases.find(canvas);
    if (!cam || it == ctx->canvases.end()) return set_error(RT_ERR_INVALID, "null camera or unknown canvas");
    const rt_context::Canvas& c = it->second;
    const size_t elem = o->out_format == RT_OUT_U8 ? 1 : (o->precision == RT_PRECISION_F32 ? 4 : 8);
    if ((uint64_t)cam->width * cam->height * 3 * elem > c.bytes || o->shard_index >= c.n_flags || seq == 0)
        return set_error(RT_ERR_INVALID, "rt_render_to_canvas: canvas too small, shard without a flag, or seq 0");
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    RT_HIP(hipSetDevice(ctx->device));
    unsigned long long* flags = canvas_flags(canvas, c.bytes);
    // the owner has released the previous frame (its readers are done)
    if (seq > 1) RT_HIP(launch_canvas_wait(flags + c.n_flags, 1, seq - 1, timeout_ticks(timeout_ms), ctx->d_error, s));
    if (cam->width && cam->height &&
        (rc = launch_frame(ctx, cam, o, o->shard_index, o->shard_count, canvas, s, true)))
        return rc;
    RT_HIP(launch_canvas_signal(flags + o->shard_index, seq, s));
    return RT_OK;
}

int rt_canvas_wait(rt_context* ctx, void* canvas, uint64_t seq, double timeout_ms, void* hip_stream) {
    if (!ctx) return set_error(RT_ERR_INVALID, "null context");
    auto it = ctx->canvases.find(canvas);
    if (it == ctx->canvases.end()) return set_error(RT_ERR_INVALID, "unknown canvas");
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(launch_canvas_wait(canvas_flags(canvas, it->second.bytes), it->second.n_flags, seq, timeout_ticks(timeout_ms),
                              ctx->d_error, static_cast<hipStream_t>(hip_stream)));
    return RT_OK;
}

int rt_canvas_read(rt_context* ctx, void* canvas, void* out_host, uint64_t bytes) {
    if (!ctx || !out_host) return set_error(RT_ERR_INVALID, "null argument");
    auto it = ctx->canvases.find(canvas);
    if (it == ctx->canvases.end() || bytes > it->second.bytes) return set_error(RT_ERR_INVALID, "unknown canvas or size");
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(hipDeviceSynchronize());
    RT_HIP(hipMemcpy(out_host, canvas, bytes, hipMemcpyDeviceToHost));
    return check_pool_error(ctx);
}

int rt_canvas_release(rt_context* ctx, void* canvas, uint64_t seq, void* hip_stream) {
    if (!ctx) return set_error(RT_ERR_INVALID, "null context");
    auto it = ctx->canvases.find(canvas);
    if (it == ctx->canvases.end()) return set_error(RT_ERR_INVALID, "unknown canvas");
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(launch_canvas_signal(canvas_flags(canvas, it->second.bytes) + it->second.n_flags, seq,
                                static_cast<hipStream_t>(hip_stream)));
    return RT_OK;
}

}  // extern "C"

namespace rtc {

}  // namespace rtc

extern "C" {

int rt_shard_rows(uint32_t height, uint32_t shard_count, uint32_t* rows) {
    if (!rows || shard_count == 0) return set_error(RT_ERR_INVALID, "bad arguments");
    *rows = tile_rows_for(height, shard_count, 0) * RT_TILE_H;
    return RT_OK;
}

int rt_shard_row_map(uint32_t height, uint32_t shard_count, uint32_t* shard_of_row, uint32_t* strip_row_of_row) {
    if (shard_count == 0 || (height && (!shard_of_row || !strip_row_of_row)))
        return set_error(RT_ERR_INVALID, "bad arguments");
    for (uint32_t y = 0; y < height; ++y) shard_of_image_row(y, shard_count, &shard_of_row[y], &strip_row_of_row[y]);
    return RT_OK;
}

int rt_render_device(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* out_device,
                     void* hip_stream) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if ((rc = check_options(o))) return rc;
    if (!cam || (!out_device && !(ctx->comm && ctx->rank != 0)))  // a group's other ranks write no image
        return set_error(RT_ERR_INVALID, "null camera or output");
    if (cam->width == 0 || cam->height == 0) return RT_OK;  // empty canvas (canvas.rs:27-35)
    hipStream_t s = static_cast<hipStream_t>(hip_stream);  // NULL = HIP's default stream
    if (ctx->comm) return group_render_device(ctx, cam, o, out_device, s);
    return launch_frame(ctx, cam, o, o->shard_index, o->shard_count, out_device, s);
}

int rt_render(rt_context* ctx, const rt_camera_desc* cam, const rt_render_options* o, void* out_host,
              rt_stats* stats) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if ((rc = check_options(o))) return rc;
    if (!cam) return set_error(RT_ERR_INVALID, "null camera");
    if (ctx->comm) return group_render(ctx, cam, o, out_host, stats);
    if (!out_host) return set_error(RT_ERR_INVALID, "null output");
    RT_HIP(hipSetDevice(ctx->device));
    const size_t elem = o->out_format == RT_OUT_U8 ? 1 : (o->precision == RT_PRECISION_F32 ? 4 : 8);
    const uint32_t rows = tile_rows_for(cam->height, o->shard_count, o->shard_index) * RT_TILE_H;
    const uint32_t valid_rows = o->shard_count == 1 ? cam->height : rows;
    const size_t bytes = (size_t)rows * cam->width * 3 * elem;
    const size_t out_bytes = (size_t)valid_rows * cam->width * 3 * elem;
    if (bytes == 0) {
        if (stats) std::memset(stats, 0, sizeof(*stats));
        return RT_OK;
    }
    InitTrace tr("rt_render");
    if ((rc = ensure_scratch(ctx, bytes))) return rc;
    tr.step("scratch");
    if ((rc = ensure_host_counters(ctx))) return rc;
    tr.step("pinned counters");
    hipStream_t s = ctx->stream;
    // counters before and after, and the error flag, come back in pinned
    // memory on the stream: one host sync for the whole frame
    if ((rc = order_after_last(ctx, s))) return rc;
    const size_t cbytes = (size_t)kCounterShards * kNumCounters * sizeof(unsigned long long);
    unsigned long long* h_before = ctx->h_counters;
    unsigned long long* h_after = ctx->h_counters + (size_t)kCounterShards * kNumCounters;
    int32_t* h_err = reinterpret_cast<int32_t*>(h_after + (size_t)kCounterShards * kNumCounters);
    RT_HIP(hipMemcpyAsync(h_before, ctx->d_counters, cbytes, hipMemcpyDeviceToHost, s));
    if (o->shard_count > 1) RT_HIP(hipMemsetAsync(ctx->d_scratch, 0, bytes, s));  // strip rows past the canvas
    RT_HIP(hipEventRecord(ctx->ev_start, s));
    tr.step("enqueue before launch");
    if ((rc = launch_frame(ctx, cam, o, o->shard_index, o->shard_count, ctx->d_scratch, s))) return rc;
    tr.step("launch");
    RT_HIP(hipEventRecord(ctx->ev_stop, s));
    RT_HIP(hipMemcpyAsync(h_after, ctx->d_counters, cbytes, hipMemcpyDeviceToHost, s));
    RT_HIP(hipMemcpyAsync(h_err, ctx->d_error, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if ((rc = copy_to_host(ctx, out_host, out_bytes))) return rc;
    tr.step("enqueue copies");
    RT_HIP(hipStreamSynchronize(s));
    tr.step("synchronize (kernel + copies)");
    float ms = 0.f;
    RT_HIP(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_stop));
    if (*h_err) {
        RT_HIP(hipMemsetAsync(ctx->d_error, 0, sizeof(int32_t), s));
        RT_HIP(hipStreamSynchronize(s));
        return set_error(RT_ERR_POOL, device_error_text(*h_err));
    }
    if (stats) {
        unsigned long long before[kNumCounters] = {}, after[kNumCounters] = {};
        for (int sh = 0; sh < kCounterShards; ++sh)
            for (int i = 0; i < kNumCounters; ++i) {
                before[i] += h_before[(size_t)sh * kNumCounters + i];
                after[i] += h_after[(size_t)sh * kNumCounters + i];
            }
        fill_stats(ctx, before, after, ms, stats);
    }
    return RT_OK;
}

int rt_color_at(rt_context* ctx, const double* rays, uint64_t n, uint32_t depth, uint32_t precision, double* out,
                rt_stats* stats) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!rays || !out) return set_error(RT_ERR_INVALID, "null rays or output");
    if (precision > RT_PRECISION_F64) return set_error(RT_ERR_INVALID, "unknown precision");
    if (depth > RT_MAX_SUPPORTED_DEPTH) return set_error(RT_ERR_INVALID, "max_depth above RT_MAX_SUPPORTED_DEPTH");
    if (n == 0) {
        if (stats) std::memset(stats, 0, sizeof(*stats));
        return RT_OK;
    }
    // Worlds with secondary rays run the pool kernel, whose fixed-point pixel
    // sums are sized for unit directions (check_pixel_range): with |d| != 1
    // the specular term grows as |d|^shininess (material.rs:100-109, eye =
    // -d) past any fixed range.  The camera's rays are unit (camera.rs:66),
    // so only a caller's own rays can be refused here.
    if ((ctx->w32.scene.any_secondary || ctx->w64.scene.any_secondary) && depth > 0) {
        for (uint64_t i = 0; i < n; ++i) {
            const double* d = rays + 6 * i + 3;
            const double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
            if (!(std::fabs(dd - 1.0) <= 1e-6))
                return set_error(RT_ERR_INVALID, "rt_color_at: ray " + std::to_string(i) + " has |d|^2 = " +
                                                     std::to_string(dd) +
                                                     "; in a world with reflective or transparent materials "
                                                     "directions must be unit length (within 1e-6)");
        }
    }
    RT_HIP(hipSetDevice(ctx->device));
    const size_t elem = precision == RT_PRECISION_F32 ? 4 : 8;
    const size_t in_bytes = n * 6 * sizeof(double), out_bytes = n * 3 * elem;
    if ((rc = ensure_scratch(ctx, in_bytes + out_bytes))) return rc;
    double* d_rays = static_cast<double*>(ctx->d_scratch);
    void* d_out = static_cast<char*>(ctx->d_scratch) + in_bytes;
    RT_HIP(hipMemcpy(d_rays, rays, in_bytes, hipMemcpyHostToDevice));
    unsigned long long before[kNumCounters], after[kNumCounters];
    if ((rc = read_counters(ctx, before))) return rc;
    RT_HIP(hipEventRecord(ctx->ev_start, ctx->stream));
    if (precision == RT_PRECISION_F32)
        rc = launch<float>(ctx, ctx->w32, nullptr, d_rays, n, depth, RT_OUT_REAL, 0, 1, d_out, ctx->stream);
    else
        rc = launch<double>(ctx, ctx->w64, nullptr, d_rays, n, depth, RT_OUT_REAL, 0, 1, d_out, ctx->stream);
    if (rc) return rc;
    RT_HIP(hipEventRecord(ctx->ev_stop, ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    float ms = 0.f;
    RT_HIP(hipEventElapsedTime(&ms, ctx->ev_start, ctx->ev_stop));
    if (precision == RT_PRECISION_F32) {
        std::vector<float> tmp(n * 3);
        RT_HIP(hipMemcpy(tmp.data(), d_out, out_bytes, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < n * 3; ++i) out[i] = tmp[i];
    } else {
        RT_HIP(hipMemcpy(out, d_out, out_bytes, hipMemcpyDeviceToHost));
    }
    if ((rc = check_pool_error(ctx))) return rc;
    if (stats) {
        if ((rc = read_counters(ctx, after))) return rc;
        fill_stats(ctx, before, after, ms, stats);
    }
    return RT_OK;
}

namespace {
// rt_debug_intersect / rt_debug_normal: one launch of the KAT harness kernel
int debug_shape(rt_context* ctx, uint32_t shape, uint32_t mode, const double* in, size_t in_stride, uint64_t n,
                uint32_t precision, uint32_t world_space, double* out, size_t out_stride) {
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!in || !out) return set_error(RT_ERR_INVALID, "null input or output");
    if (precision > RT_PRECISION_F64) return set_error(RT_ERR_INVALID, "unknown precision");
    if (shape >= ctx->world_slot.size()) return set_error(RT_ERR_INVALID, "shape index out of range");
    if (n == 0) return RT_OK;
    if (n > 0xFFFFFFFFull) return set_error(RT_ERR_INVALID, "too many rays");
    RT_HIP(hipSetDevice(ctx->device));
    const size_t in_bytes = n * in_stride * sizeof(double), out_bytes = n * out_stride * sizeof(double);
    if ((rc = ensure_scratch(ctx, in_bytes + out_bytes))) return rc;
    double* d_in = static_cast<double*>(ctx->d_scratch);
    double* d_out = d_in + n * in_stride;
    RT_HIP(hipMemcpyAsync(d_in, in, in_bytes, hipMemcpyHostToDevice, ctx->stream));
    const int32_t ws = ctx->world_slot[shape];
    const int slot = ws & 0xFFFFFF, kind = ws >> 24;
    if ((rc = order_after_last(ctx, ctx->stream))) return rc;
    hipError_t e = precision == RT_PRECISION_F32
                       ? launch_debug_shape<float>(ctx->w32.shapes, slot, kind, mode, world_space, d_in, (uint32_t)n,
                                                   d_out, ctx->stream)
                       : launch_debug_shape<double>(ctx->w64.shapes, slot, kind, mode, world_space, d_in, (uint32_t)n,
                                                    d_out, ctx->stream);
    if (e != hipSuccess) return set_error(RT_ERR_HIP, std::string("debug_shape launch: ") + hipGetErrorString(e));
    RT_HIP(hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}
}  // namespace

int rt_debug_intersect(rt_context* ctx, uint32_t shape, const double* rays, uint64_t n, uint32_t precision,
                       uint32_t world_space, double* out) {
    return debug_shape(ctx, shape, 0, rays, 6, n, precision, world_space, out, 1 + RT_DEBUG_MAX_ENTRIES);
}

int rt_debug_normal(rt_context* ctx, uint32_t shape, const double* points, uint64_t n, uint32_t precision,
                    uint32_t world_space, double* out) {
    return debug_shape(ctx, shape, 1, points, 3, n, precision, world_space, out, 3);
}

int rt_context_set_frames_in_flight(rt_context* ctx, uint32_t frames) {
    if (!ctx || frames < 1) return set_error(RT_ERR_INVALID, "bad arguments");
    // (an A/B setting of RTC_DEBUG wins over the hint)
    std::string v;
    const bool grid_knob = debug_knob("direct_oversub", &v), split_knob = debug_knob("split", &v);
    std::vector<rt_context*> ms{ctx};
    ms.insert(ms.end(), ctx->peers.begin(), ctx->peers.end());
    for (rt_context* m : ms) {
        if (!grid_knob) m->direct_oversub10 = frames > 1 ? 15u : 25u;
        // pool kernels: with the next frame filling a launch's tail, tiles
        // split only above 1.5x the mean workgroup load (a 4K shard of 8 with
        // two in flight, round 6: cover 0.104 -> 0.094 ms per frame, table
        // 0.115 -> 0.113; a frame alone keeps 1.0x)
        const double split = frames > 1 ? 1.5 : 1.0;
        if (!split_knob && m->split_factor != split) {
            m->split_factor = split;
            m->order_valid = false;  // the next launches rebuild the tile order with it
        }
    }
    return RT_OK;
}

int rt_context_set_jit(rt_context* ctx, int mode) {
    if (!ctx || mode < RT_JIT_OFF || mode > RT_JIT_EAGER) return set_error(RT_ERR_INVALID, "bad arguments");
    ctx->jit_mode = mode;
    for (rt_context* p : ctx->peers) p->jit_mode = mode;
    return RT_OK;
}

int rt_jit_status(rt_context* ctx, int* used_last_launch, double* compile_ms, char* log, size_t log_len) {
    if (!ctx) return set_error(RT_ERR_INVALID, "null context");
    if (used_last_launch) *used_last_launch = ctx->jit_used ? 1 : 0;
    if (compile_ms) *compile_ms = ctx->jit_compile_ms;
    if (log && log_len) {
        std::strncpy(log, ctx->jit_log.c_str(), log_len - 1);
        log[log_len - 1] = '\0';
    }
    return RT_OK;
}

int rt_jit_wait(rt_context* ctx, double timeout_ms, int* pending) {
    if (!ctx) return set_error(RT_ERR_INVALID, "null context");
    // one deadline for the whole group: each member waits for what is left of it
    const auto t0 = std::chrono::steady_clock::now();
    auto remaining = [&] {
        if (timeout_ms < 0) return timeout_ms;
        const double spent = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return std::max(0.0, timeout_ms - spent);
    };
    int total = 0, left = 0;
    for (rt_context* c : ctx->peers) {
        jit_wait(c, remaining(), &left);
        total += left;
    }
    jit_wait(ctx, remaining(), &left);
    if (pending) *pending = total + left;
    return RT_OK;
}

int rt_debug_stamps(rt_context* ctx, uint64_t* out, uint32_t max_wg, uint32_t* n) {
    if (!ctx || !n) return set_error(RT_ERR_INVALID, "null argument");
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(hipDeviceSynchronize());
    *n = ctx->stamp_count;
    const uint32_t copy = std::min(max_wg, ctx->stamp_count);
    if (out && copy)
        RT_HIP(hipMemcpy(out, ctx->d_stamps, 2 * sizeof(uint64_t) * copy, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_item_log(rt_context* ctx, uint64_t* out, uint32_t max_items, uint32_t* n) {
    if (!ctx || !n) return set_error(RT_ERR_INVALID, "null argument");
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(hipDeviceSynchronize());
    uint64_t count = 0;
    if (ctx->d_item_log) RT_HIP(hipMemcpy(&count, ctx->d_item_log, sizeof count, hipMemcpyDeviceToHost));
    *n = (uint32_t)std::min<uint64_t>(count, ctx->item_log_capacity);
    const uint32_t copy = std::min(max_items, *n);
    if (out && copy)
        RT_HIP(hipMemcpy(out, ctx->d_item_log + 1, 3 * sizeof(uint64_t) * copy, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_tile_costs(rt_context* ctx, uint32_t* out, uint32_t max_tiles, uint32_t* n) {
    if (!ctx || !n) return set_error(RT_ERR_INVALID, "null argument");
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(hipDeviceSynchronize());
    *n = ctx->order_valid ? ctx->order_capacity : 0;
    const uint32_t copy = std::min(max_tiles, *n);
    if (out && copy) RT_HIP(hipMemcpy(out, ctx->d_tile_cost, copy * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_read_counters(rt_context* ctx, rt_stats* totals) {
    if (!ctx || !totals) return set_error(RT_ERR_INVALID, "null argument");
    if (!ctx->peers.empty()) return group_read_counters(ctx, totals);
    RT_HIP(hipSetDevice(ctx->device));
    RT_HIP(hipDeviceSynchronize());
    unsigned long long zero[kNumCounters] = {}, now[kNumCounters];
    int rc = read_counters(ctx, now);
    if (rc) return rc;
    fill_stats(ctx, zero, now, 0.f, totals);
    return check_pool_error(ctx);
}

int rt_read_generation_counts(rt_context* ctx, rt_generation_counts* out) {
    if (!ctx || !out) return set_error(RT_ERR_INVALID, "null argument");
    std::memset(out, 0, sizeof(*out));
    std::vector<rt_context*> members = {ctx};
    members.insert(members.end(), ctx->peers.begin(), ctx->peers.end());
    for (rt_context* m : members) {
        unsigned long long buf[2 * kGenSlots];
        RT_HIP(hipSetDevice(m->device));
        RT_HIP(hipDeviceSynchronize());
        RT_HIP(hipMemcpy(buf, m->d_gen_counts, sizeof buf, hipMemcpyDeviceToHost));
        for (int i = 0; i < kGenSlots; ++i) {
            out->traced[i] += buf[i];
            out->shaded[i] += buf[kGenSlots + i];
        }
    }
    RT_HIP(hipSetDevice(ctx->device));
    return RT_OK;
}

int rt_assemble_shards(rt_context* ctx, const void* gathered, uint32_t width, uint32_t height, uint32_t shards,
                       uint32_t bpp, void* image, void* hip_stream) {
    if (!ctx || !gathered || !image || shards == 0 || bpp == 0) return set_error(RT_ERR_INVALID, "bad arguments");
    RT_HIP(hipSetDevice(ctx->device));
    uint32_t rows = 0;
    rt_shard_rows(height, shards, &rows);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);  // NULL = HIP's default stream
    RT_HIP(launch_assemble(gathered, image, width, height, shards, rows, bpp, s));
    return RT_OK;
}

}  // extern "C"
