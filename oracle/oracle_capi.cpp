// oracle_capi.cpp — TEST INFRASTRUCTURE.  C entry points of the f64 oracle
// (rtc_oracle.hpp) over the same POD descriptors the product C-ABI takes
// (include/rtc.h), so tests/ and bench.py's cpu_baseline leg can render the
// exact world the GPU renders.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline use this library, and only as the checker.
#include <cstring>
#include <stdexcept>
#include <string>

#include "../include/rtc.h"
#include "rtc_oracle.hpp"

using namespace orc;

namespace {

M4 mat_from(const double* m) {
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.m[i][j] = m[4 * i + j];
    return r;
}

// Build the trait-object world the reference would hold for these tables.
World build_world(const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
                  const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights, uint32_t nl) {
    std::vector<PatternPtr> pp(np);
    for (uint32_t i = 0; i < np; ++i) pp[i] = std::make_shared<Pattern>();
    for (uint32_t i = 0; i < np; ++i) {
        const rt_pattern_desc& d = pats[i];
        Pattern& p = *pp[i];
        p.kind = d.kind;
        p.a = {d.color_a[0], d.color_a[1], d.color_a[2]};
        p.b = {d.color_b[0], d.color_b[1], d.color_b[2]};
        p.inv = mat_from(d.inverse);
        if (d.kind == RT_PATTERN_COMPLEX) {
            if (d.sub_a < 0 || d.sub_b < 0 || (uint32_t)d.sub_a >= np || (uint32_t)d.sub_b >= np)
                throw std::runtime_error("complex pattern sub-pattern index out of range");
            p.sub_a = pp[d.sub_a];
            p.sub_b = pp[d.sub_b];
        }
    }
    World w;
    for (uint32_t i = 0; i < nl; ++i)
        w.lights.push_back({{lights[i].position[0], lights[i].position[1], lights[i].position[2]},
                            {lights[i].intensity[0], lights[i].intensity[1], lights[i].intensity[2]}});
    w.shapes.reserve(ns);
    for (uint32_t i = 0; i < ns; ++i) {
        const rt_shape_desc& d = shapes[i];
        if (d.material < 0 || (uint32_t)d.material >= nm) throw std::runtime_error("material index out of range");
        const rt_material_desc& md = mats[d.material];
        Shape s;
        s.kind = d.kind;
        s.inv = mat_from(d.inverse);
        s.minimum = d.minimum;
        s.maximum = d.maximum;
        s.closed = d.closed != 0;
        s.v1 = {d.vertex_1[0], d.vertex_1[1], d.vertex_1[2]};
        s.e1 = {d.edge_1[0], d.edge_1[1], d.edge_1[2]};
        s.e2 = {d.edge_2[0], d.edge_2[1], d.edge_2[2]};
        s.tn = {d.normal[0], d.normal[1], d.normal[2]};
        s.v2 = add(s.v1, s.e1);
        s.v3 = add(s.v1, s.e2);
        Material& m = s.material;
        m.color = {md.color[0], md.color[1], md.color[2]};
        m.ambient = md.ambient;
        m.diffuse = md.diffuse;
        m.specular = md.specular;
        m.shininess = md.shininess;
        m.reflectiveness = md.reflectiveness;
        m.transparency = md.transparency;
        m.refractive_index = md.refractive_index;
        m.casts_shadow = md.casts_shadow != 0;
        if (md.pattern >= 0) {
            if ((uint32_t)md.pattern >= np) throw std::runtime_error("pattern index out of range");
            m.pattern = pp[md.pattern];
        }
        w.shapes.push_back(s);
    }
    return w;
}

Camera camera_from(const rt_camera_desc& c) {
    Camera cam;
    cam.hsize = c.width;
    cam.vsize = c.height;
    cam.fov = c.field_of_view;
    cam.half_width = c.half_width;
    cam.half_height = c.half_height;
    cam.pixel_size = c.pixel_size;
    cam.inv = mat_from(c.inverse);
    cam.origin = {c.origin[0], c.origin[1], c.origin[2]};
    return cam;
}

void fill_stats(const Counters& k, rt_stats* s) {
    if (!s) return;
    std::memset(s, 0, sizeof(*s));
    s->primary = k.primary;
    s->shadow = k.shadow;
    s->reflect = k.reflect;
    s->refract = k.refract;
    s->shaded = k.shaded;
    s->lit_patterned = k.lit_patterned;
    s->refract_evals = k.refract_evals;
    s->schlick_evals = k.schlick_evals;
}

thread_local std::string g_err;
thread_local Counters g_last;  // counters of this thread's last render / color_at (orc_last_generations)

}  // namespace

extern "C" {

const char* orc_last_error(void) { return g_err.c_str(); }

// Camera::new + set_transformation(view_transform(from, to, up)) — the
// scene_loader.rs:265-266 sequence — restated independently of the product.
int orc_camera(uint32_t width, uint32_t height, double fov, const double* from, const double* to, const double* up,
               rt_camera_desc* out) {
    Camera c(width, height, fov);
    c.set_transformation(view_transform({from[0], from[1], from[2]}, {to[0], to[1], to[2]}, {up[0], up[1], up[2]}));
    out->width = width;
    out->height = height;
    out->field_of_view = fov;
    out->half_width = c.half_width;
    out->half_height = c.half_height;
    out->pixel_size = c.pixel_size;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out->inverse[4 * i + j] = c.inv.m[i][j];
    out->origin[0] = c.origin.x;
    out->origin[1] = c.origin.y;
    out->origin[2] = c.origin.z;
    return 0;
}

// Matrix<4>::inverse (matrix.rs:247-258)
int orc_inverse(const double* m, double* out) {
    M4 r = inverse(mat_from(m));
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = r.m[i][j];
    return 0;
}

// Camera::render (threads <= 1) / render_parallel: rows [row_begin, row_end).
int orc_render(const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
               const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights, uint32_t nl,
               const rt_camera_desc* cam, uint32_t depth, uint32_t row_begin, uint32_t row_end, int threads,
               double* out, rt_stats* stats) {
    try {
        if (!cam || !out || row_end > cam->height || row_begin > row_end) throw std::runtime_error("bad arguments");
        World w = build_world(shapes, ns, mats, nm, pats, np, lights, nl);
        Counters k;
        render_rows(camera_from(*cam), w, (int)depth, row_begin, row_end, threads, out, &k);
        fill_stats(k, stats);
        g_last = k;
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// World::color_at for a batch of rays {ox,oy,oz,dx,dy,dz}.
int orc_color_at(const rt_shape_desc* shapes, uint32_t ns, const rt_material_desc* mats, uint32_t nm,
                 const rt_pattern_desc* pats, uint32_t np, const rt_light_desc* lights, uint32_t nl,
                 const double* rays, uint64_t n, uint32_t depth, double* out, rt_stats* stats) {
    try {
        World w = build_world(shapes, ns, mats, nm, pats, np, lights, nl);
        Counters k;
        Hits xs;
        for (uint64_t i = 0; i < n; ++i) {
            const double* r = rays + 6 * i;
            k.primary++;
            Color c = w.color_at(Ray{{r[0], r[1], r[2]}, {r[3], r[4], r[5]}}, xs, (int)depth, &k);
            out[3 * i + 0] = c.r;
            out[3 * i + 1] = c.g;
            out[3 * i + 2] = c.b;
        }
        fill_stats(k, stats);
        g_last = k;
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Per-generation counts of this thread's last orc_render / orc_color_at,
// indexed by `remaining` (Counters::traced_at / shaded_at): 17 entries each.
int orc_last_generations(uint64_t* traced, uint64_t* shaded) {
    for (int i = 0; i <= Counters::kMaxRemaining; ++i) {
        traced[i] = g_last.traced_at[i];
        shaded[i] = g_last.shaded_at[i];
    }
    return 0;
}

}  // extern "C"
