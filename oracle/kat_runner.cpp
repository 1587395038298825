// kat_runner.cpp — TEST INFRASTRUCTURE.  Re-enacts the reference's own unit
// tests (the scenarios of ray-tracer/src/**/*.rs `#[cfg(test)]` modules) on
// the f64 oracle and prints every computed value as JSON.  The expected
// values live in tests/golden/reference_kats.json (transcribed from the
// reference test assertions, with file:line), compared by
// tests/test_oracle_kat.py.  This pins the oracle before it is trusted.
#include <cstdio>
#include <string>
#include <vector>

#include "rtc_oracle.hpp"

using namespace orc;

static bool first_case = true;
static void emit(const std::string& name, const std::vector<double>& v) {
    std::printf("%s\n  \"%s\": [", first_case ? "{" : ",", name.c_str());
    first_case = false;
    for (size_t i = 0; i < v.size(); ++i) std::printf("%s%.17g", i ? ", " : "", v[i]);
    std::printf("]");
}
static std::vector<double> vv(const V3& a) { return {a.x, a.y, a.z}; }
static std::vector<double> cv(const Color& a) { return {a.r, a.g, a.b}; }
static std::vector<double> mv(const M4& m) {
    std::vector<double> r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.push_back(m.m[i][j]);
    return r;
}
static std::vector<double> ts(const Hits& xs) {
    std::vector<double> r;
    for (auto& h : xs) r.push_back(h.t);
    return r;
}
static Hits local(const Shape& s, const Point& o, const Vector& d) {
    Hits xs;
    local_intersect(s, Ray{o, d}, xs);
    return xs;
}
static Hits world_ray(const Shape& s, const Point& o, const Vector& d) {  // Ray::intersect, ray.rs:35-42
    Hits xs;
    local_intersect(s, transform(Ray{o, d}, s.inv), xs);
    return xs;
}
static const double S2 = std::sqrt(2.0);

int main() {
    // ------------------------------------------------------------ camera.rs
    emit("camera.pixel_size_horizontal", {Camera(200, 125, PI / 2.0).pixel_size});
    emit("camera.pixel_size_vertical", {Camera(125, 200, PI / 2.0).pixel_size});
    {
        Camera c(201, 101, PI / 2.0);
        Ray r = c.ray_for_pixel(100, 50);
        auto v = vv(r.origin);
        auto d = vv(r.direction);
        v.insert(v.end(), d.begin(), d.end());
        emit("camera.ray_through_center", v);
        r = c.ray_for_pixel(0, 0);
        v = vv(r.origin);
        d = vv(r.direction);
        v.insert(v.end(), d.begin(), d.end());
        emit("camera.ray_through_corner", v);
        c.set_transformation(mul(rotation_y(PI / 4.0), translation(0, -2, 5)));
        r = c.ray_for_pixel(100, 50);
        v = vv(r.origin);
        d = vv(r.direction);
        v.insert(v.end(), d.begin(), d.end());
        emit("camera.ray_transformed_camera", v);
    }
    {
        World w = default_world();
        Camera c(11, 11, PI / 2.0);
        c.set_transformation(view_transform({0, 0, -5}, {0, 0, 0}, {0, 1, 0}));
        std::vector<double> img(11 * 11 * 3);
        render_rows(c, w, World::MAX_REFLECTION_ITERATIONS, 0, 11, 1, img.data(), nullptr);
        size_t i = 3 * (5 + 5 * 11);
        emit("camera.render_default_world", {img[i], img[i + 1], img[i + 2]});
        render_rows(c, w, World::MAX_REFLECTION_ITERATIONS, 0, 11, 4, img.data(), nullptr);
        emit("camera.render_parallel_default_world", {img[i], img[i + 1], img[i + 2]});
    }

    // ------------------------------------------------------------- world.rs
    {
        World w = default_world();
        Hits xs;
        w.collect_intersections(Ray{{0, 0, -5}, {0, 0, 1}}, xs);
        emit("world.intersect_world_with_ray", ts(xs));
    }
    {
        World w = default_world();
        Ray r{{0, 0, -5}, {0, 0, 1}};
        Hits none, buf;
        Comps c = prepare_computations({4.0, &w.shapes[0]}, r, none);
        emit("world.shading_intersection", cv(w.shade_hit(c, buf, 1)));
    }
    {
        World w = default_world();
        w.lights = {{{0, 0.25, 0}, WHITE}};
        Ray r{{0, 0, 0}, {0, 0, 1}};
        Hits none, buf;
        Comps c = prepare_computations({0.5, &w.shapes[1]}, r, none);
        emit("world.shading_intersection_from_inside", cv(w.shade_hit(c, buf, 1)));
    }
    {
        World w = default_world();
        Hits xs;
        emit("world.color_when_ray_misses", cv(w.color_at(Ray{{0, 0, -5}, {0, 1, 0}}, xs)));
        emit("world.color_when_ray_hits", cv(w.color_at(Ray{{0, 0, -5}, {0, 0, 1}}, xs)));
    }
    {
        World w = default_world();
        w.shapes[0].material.ambient = 1.0;
        w.shapes[1].material.ambient = 1.0;
        Hits xs;
        emit("world.color_with_intersection_behind_ray", cv(w.color_at(Ray{{0, 0, 0.75}, {0, 0, -1}}, xs)));
    }
    {
        World w = default_world();
        Hits xs;
        emit("world.shadow_predicates", {(double)w.is_in_shadow(w.lights[0], {0, 10, 0}, xs),
                                         (double)w.is_in_shadow(w.lights[0], {-20, 20, -20}, xs),
                                         (double)w.is_in_shadow(w.lights[0], {-2, 2, -2}, xs),
                                         (double)w.is_in_shadow(w.lights[0], {10, -10, 10}, xs)});
    }
    {
        World w = default_world();
        w.lights = {{{0, 0, -10}, WHITE}};
        w.shapes.push_back(Shape());
        Shape s2;
        s2.set_transformation(translation(0, 0, 10));
        w.shapes.push_back(s2);
        Shape boxed = s2;
        Hits none, buf;
        Comps c = prepare_computations({4.0, &boxed}, Ray{{0, 0, 5}, {0, 0, 1}}, none);
        emit("world.shade_hit_in_shadow", cv(w.shade_hit(c, buf, 1)));
    }
    {
        World w = default_world();
        Shape s = w.shapes[1];
        s.material.ambient = 1.0;
        w.shapes[0] = s;
        Hits none, buf;
        Comps c = prepare_computations({1.0, &w.shapes[1]}, Ray{{0, 0, 0}, {0, 0, 1}}, none);
        emit("world.reflected_color_nonreflective", cv(w.reflected_color(c, buf, 1)));
    }
    auto reflective_plane_world = [](World& w, Shape& plane) {
        plane.kind = S_PLANE;
        plane.material.reflectiveness = 0.5;
        plane.set_transformation(translation(0, -1, 0));
        w.shapes.push_back(plane);
    };
    {
        World w = default_world();
        Shape p;
        reflective_plane_world(w, p);
        Hits none, buf;
        Ray r{{0, 0, -3}, {0, -S2 / 2.0, S2 / 2.0}};
        Comps c = prepare_computations({S2, &p}, r, none);
        emit("world.reflected_color_reflective", cv(w.reflected_color(c, buf, 1)));
        emit("world.shade_hit_reflective", cv(w.shade_hit(c, buf, 1)));
        emit("world.reflected_color_at_max_depth", cv(w.reflected_color(c, buf, 0)));
    }
    {
        World w;
        w.lights = {{{0, 0, 0}, WHITE}};
        Shape lower, upper;
        lower.kind = upper.kind = S_PLANE;
        lower.material.reflectiveness = upper.material.reflectiveness = 1.0;
        lower.set_transformation(translation(0, -1, 0));
        upper.set_transformation(translation(0, 1, 0));
        w.shapes = {lower, upper};
        Hits xs;
        emit("world.no_infinite_recursion", cv(w.color_at(Ray{{0, 0, 0}, {0, 1, 0}}, xs)));
    }
    {
        World w = default_world();
        Hits xs{{4.0, &w.shapes[0]}, {6.0, &w.shapes[0]}}, buf;
        Comps c = prepare_computations(xs[0], Ray{{0, 0, -5}, {0, 0, 1}}, xs);
        emit("world.refracted_color_opaque", cv(w.refracted_color(c, buf, 5)));
    }
    {
        World w = default_world();
        w.shapes[0].material.transparency = 1.0;
        w.shapes[0].material.refractive_index = 1.5;
        Shape boxed = w.shapes[0];
        Hits xs{{4.0, &boxed}, {6.0, &boxed}}, buf;
        Comps c = prepare_computations(xs[0], Ray{{0, 0, -5}, {0, 0, 1}}, xs);
        emit("world.refracted_color_at_max_depth", cv(w.refracted_color(c, buf, 0)));
        Hits ys{{-S2 / 2.0, &boxed}, {S2 / 2.0, &boxed}};
        Comps d = prepare_computations(ys[1], Ray{{0, 0, S2 / 2.0}, {0, 1, 0}}, ys);
        emit("world.refracted_color_total_internal_reflection", cv(w.refracted_color(d, buf, 5)));
    }
    {
        World w = default_world();
        w.shapes[0].material.ambient = 1.0;
        auto tp = std::make_shared<Pattern>();
        tp->kind = P_TEST;
        w.shapes[0].material.pattern = tp;
        w.shapes[1].material.transparency = 1.0;
        w.shapes[1].material.refractive_index = 1.5;
        Hits xs{{-0.9899, &w.shapes[0]}, {-0.4899, &w.shapes[1]}, {0.4899, &w.shapes[1]}, {0.9899, &w.shapes[0]}},
            buf;
        Comps c = prepare_computations(xs[2], Ray{{0, 0, 0.1}, {0, 1, 0}}, xs);
        emit("world.refracted_color_with_refracted_ray", cv(w.refracted_color(c, buf, 5)));
    }
    for (int both = 0; both < 2; ++both) {
        World w = default_world();
        Shape floor;
        floor.kind = S_PLANE;
        floor.material.transparency = 0.5;
        floor.material.refractive_index = 1.5;
        if (both) floor.material.reflectiveness = 0.5;
        floor.set_transformation(translation(0, -1, 0));
        w.shapes.push_back(floor);
        Shape ball;
        ball.material.color = {1, 0, 0};
        ball.material.ambient = 0.5;
        ball.set_transformation(translation(0, -3.5, -0.5));
        w.shapes.push_back(ball);
        Shape boxed = floor;
        Hits xs{{S2, &boxed}}, buf;
        Comps c = prepare_computations(xs[0], Ray{{0, 0, -3}, {0, -S2 / 2.0, S2 / 2.0}}, xs);
        emit(both ? "world.shade_hit_reflective_transparent" : "world.shade_hit_transparent",
             cv(w.shade_hit(c, buf, 5)));
    }

    // ------------------------------------------------------ intersection.rs
    {
        Shape s;
        Hits none;
        Comps c = prepare_computations({4.0, &s}, Ray{{0, 0, -5}, {0, 0, 1}}, none);
        auto v = vv(c.point), e = vv(c.eye), n = vv(c.normal);
        v.insert(v.end(), e.begin(), e.end());
        v.insert(v.end(), n.begin(), n.end());
        v.push_back((double)c.inside);
        emit("intersection.precomputing_state_outside", v);
        Comps d = prepare_computations({1.0, &s}, Ray{{0, 0, 0}, {0, 0, 1}}, none);
        v = vv(d.point);
        e = vv(d.eye);
        n = vv(d.normal);
        v.insert(v.end(), e.begin(), e.end());
        v.insert(v.end(), n.begin(), n.end());
        v.push_back((double)d.inside);
        emit("intersection.precomputing_state_inside", v);
    }
    {
        Shape s;
        s.set_transformation(translation(0, 0, 1));
        Hits none;
        Comps c = prepare_computations({5.0, &s}, Ray{{0, 0, -5}, {0, 0, 1}}, none);
        emit("intersection.hit_offsets_point", {c.over_point.z, c.point.z});
        Shape g = s;
        g.material = Material::glass();
        Hits xs{{5.0, &g}};
        Comps d = prepare_computations(xs[0], Ray{{0, 0, -5}, {0, 0, 1}}, xs);
        emit("intersection.under_point_below_surface", {d.under_point.z, d.point.z});
    }
    {
        Shape p;
        p.kind = S_PLANE;
        Hits none;
        Comps c = prepare_computations({S2, &p}, Ray{{0, 1, -1}, {0, -S2 / 2.0, S2 / 2.0}}, none);
        emit("intersection.reflection_vector", vv(c.reflectv));
    }
    {
        Shape a, b, c;
        a.material = b.material = c.material = Material::glass();
        a.set_transformation(scaling(2, 2, 2));
        a.material.refractive_index = 1.5;
        b.set_transformation(translation(0, 0, -0.25));
        b.material.refractive_index = 2.0;
        c.set_transformation(translation(0, 0, 0.25));
        c.material.refractive_index = 2.5;
        Hits xs{{2, &a}, {2.75, &b}, {3.25, &c}, {4.75, &b}, {5.25, &c}, {6, &a}};
        std::vector<double> n1, n2;
        for (auto& x : xs) {
            Comps k = prepare_computations(x, Ray{{0, 0, -4}, {0, 0, 1}}, xs);
            n1.push_back(k.n1);
            n2.push_back(k.n2);
        }
        emit("intersection.refractive_indexes_n1", n1);
        emit("intersection.refractive_indexes_n2", n2);
    }

    // ------------------------------------------------------ computed_hit.rs
    {
        Shape s;
        s.material = Material::glass();
        Hits xs{{-S2 / 2.0, &s}, {S2 / 2.0, &s}};
        Comps c = prepare_computations(xs[1], Ray{{0, 0, S2 / 2.0}, {0, 1, 0}}, xs);
        Hits ys{{-1, &s}, {1, &s}};
        Comps d = prepare_computations(ys[1], Ray{{0, 0, 0}, {0, 1, 0}}, ys);
        Hits zs{{1.8589, &s}};
        Comps e = prepare_computations(zs[0], Ray{{0, 0.99, -2}, {0, 0, 1}}, zs);
        emit("computed_hit.schlick_exact", {schlick(c), schlick(d)});
        emit("computed_hit.schlick_small_angle", {schlick(e)});
    }

    // ---------------------------------------------------------- material.rs
    {
        Shape s;
        auto L = [&](Vector eye, Point lp, bool sh) {
            return cv(lighting(s.material, s, Light{lp, WHITE}, {0, 0, 0}, eye, {0, 0, -1}, sh));
        };
        emit("material.lighting_eye_between", L({0, 0, -1}, {0, 0, -10}, false));
        emit("material.lighting_eye_offset_45", L({0, S2 / 2.0, -S2 / 2.0}, {0, 0, -10}, false));
        emit("material.lighting_light_offset_45", L({0, 0, -1}, {0, 10, -10}, false));
        emit("material.lighting_eye_in_reflection", L({0, -S2 / 2.0, -S2 / 2.0}, {0, 10, -10}, false));
        emit("material.lighting_light_behind", L({0, 0, -1}, {0, 0, 10}, false));
        emit("material.lighting_in_shadow", L({0, 0, -1}, {0, 0, -10}, true));
    }

    // ---------------------------------------------------------------- shapes
    {
        Shape s;
        const double t3 = std::sqrt(3.0) / 3.0;
        std::vector<double> v;
        for (V3 p : {V3{1, 0, 0}, V3{0, 1, 0}, V3{0, 0, 1}, V3{t3, t3, t3}}) {
            auto n = vv(normal_at(s, p));
            v.insert(v.end(), n.begin(), n.end());
        }
        emit("sphere.normals", v);
        emit("sphere.normal_is_normalized", vv(normalized(normal_at(s, {t3, t3, t3}))));
        Shape t;
        t.set_transformation(translation(0, 1, 0));
        emit("sphere.normal_translated", vv(normal_at(t, {0.0, 1.0 + M_SQRT1_2, -M_SQRT1_2})));
        Shape u;
        u.set_transformation(mul(scaling(1, 0.5, 1), rotation_z(PI / 5.0)));
        emit("sphere.normal_transformed", vv(normal_at(u, {0, S2 / 2.0, -S2 / 2.0})));
    }
    {
        Shape s;
        emit("ray.sphere_middle", ts(world_ray(s, {0, 0, -5}, {0, 0, 1})));
        emit("ray.sphere_tangent", ts(world_ray(s, {0, 1, -5}, {0, 0, 1})));
        emit("ray.sphere_miss", ts(world_ray(s, {0, 2, -5}, {0, 0, 1})));
        emit("ray.sphere_inside", ts(world_ray(s, {0, 0, 0}, {0, 0, 1})));
        emit("ray.sphere_behind", ts(world_ray(s, {0, 0, 5}, {0, 0, 1})));
        Shape sc;
        sc.set_transformation(scaling(2, 2, 2));
        emit("ray.sphere_scaled", ts(world_ray(sc, {0, 0, -5}, {0, 0, 1})));
        Shape tr;
        tr.set_transformation(translation(5, 0, 0));
        emit("ray.sphere_translated", ts(world_ray(tr, {0, 0, -5}, {0, 0, 1})));
        Ray r = transform(Ray{{1, 2, 3}, {0, 1, 0}}, translation(3, 4, 5));
        auto v = vv(r.origin), d = vv(r.direction);
        v.insert(v.end(), d.begin(), d.end());
        emit("ray.translation", v);
        r = transform(Ray{{1, 2, 3}, {0, 1, 0}}, scaling(2, 3, 4));
        v = vv(r.origin);
        d = vv(r.direction);
        v.insert(v.end(), d.begin(), d.end());
        emit("ray.scaling", v);
        Ray q{{2, 3, 4}, {1, 0, 0}};
        std::vector<double> ps;
        for (double t : {0.0, 1.0, -1.0, 2.5}) {
            auto p = vv(position(q, t));
            ps.insert(ps.end(), p.begin(), p.end());
        }
        emit("ray.position", ps);
    }
    {
        Shape p;
        p.kind = S_PLANE;
        std::vector<double> v;
        for (V3 pt : {V3{0, 0, 0}, V3{10, 0, -10}, V3{-5, 0, 150}}) {
            auto n = vv(normal_at(p, pt));
            v.insert(v.end(), n.begin(), n.end());
        }
        emit("plane.normal_is_constant", v);
        emit("plane.parallel", ts(local(p, {0, 10, 0}, {0, 0, 1})));
        emit("plane.from_above", ts(local(p, {0, 1, 0}, {0, -1, 0})));
        emit("plane.from_below", ts(local(p, {0, -1, 0}, {0, 1, 0})));
    }
    {
        Shape c;
        c.kind = S_CUBE;
        struct Case { V3 o, d; };
        std::vector<Case> hits = {{{5, 0.5, 0}, {-1, 0, 0}}, {{-5, 0.5, 0}, {1, 0, 0}}, {{0.5, 5, 0}, {0, -1, 0}},
                                  {{0.5, -5, 0}, {0, 1, 0}}, {{0.5, 0, 5}, {0, 0, -1}}, {{0.5, 0, -5}, {0, 0, 1}},
                                  {{0, 0.5, 0}, {0, 0, 1}}};
        std::vector<double> v;
        for (auto& k : hits) {
            auto t = ts(local(c, k.o, k.d));
            v.push_back((double)t.size());
            v.insert(v.end(), t.begin(), t.end());
        }
        emit("cube.ray_intersects", v);
        std::vector<Case> misses = {{{-2, 0, 0}, {0.2673, 0.5345, 0.8018}}, {{0, -2, 0}, {0.8018, 0.2673, 0.5345}},
                                    {{0, 0, -2}, {0.5345, 0.8018, 0.2673}}, {{2, 0, 2}, {0, 0, -1}},
                                    {{0, 2, 2}, {0, -1, 0}}, {{2, 2, 0}, {-1, 0, 0}}, {{0, 0, 2}, {0, 0, 1}}};
        v.clear();
        for (auto& k : misses) v.push_back((double)local(c, k.o, k.d).size());
        emit("cube.ray_misses_counts", v);
        v.clear();
        for (V3 p : {V3{1, 0.5, -0.8}, V3{-1, -0.2, 0.9}, V3{-0.4, 1, -0.1}, V3{0.3, -1, -0.7}, V3{-0.6, 0.3, 1},
                     V3{0.4, 0.4, -1}, V3{1, 1, 1}, V3{-1, -1, -1}}) {
            auto n = vv(local_normal_at(c, p));
            v.insert(v.end(), n.begin(), n.end());
        }
        emit("cube.normals", v);
    }
    {
        Shape c;
        c.kind = S_CYLINDER;
        struct Case { V3 o, d; };
        std::vector<double> v;
        for (auto k : std::vector<Case>{{{1, 0, 0}, {0, 1, 0}}, {{0, 1, 0}, {0, 1, 0}}, {{0, 0, -5}, {1, 1, 1}}})
            v.push_back((double)local(c, k.o, normalized(k.d)).size());
        emit("cylinder.misses_counts", v);
        v.clear();
        for (auto k : std::vector<Case>{{{1, 0, -5}, {0, 0, 1}}, {{0, 0, -5}, {0, 0, 1}}, {{0.5, 0, -5}, {0.1, 1, 1}}}) {
            auto t = ts(local(c, k.o, normalized(k.d)));
            v.push_back((double)t.size());
            v.insert(v.end(), t.begin(), t.end());
        }
        emit("cylinder.intersects", v);
        v.clear();
        for (V3 p : {V3{1, 0, 0}, V3{0, 5, -1}, V3{0, -2, 1}, V3{-1, 1, 0}}) {
            auto n = vv(local_normal_at(c, p));
            v.insert(v.end(), n.begin(), n.end());
        }
        emit("cylinder.normals", v);
        Shape k1 = c;
        k1.minimum = 1.0;
        k1.maximum = 2.0;
        v.clear();
        for (auto k : std::vector<Case>{{{0, 1.5, 0}, {0.1, 1, 0}}, {{0, 3, -5}, {0, 0, 1}}, {{0, 0, -5}, {0, 0, 1}},
                                        {{0, 2, -5}, {0, 0, 1}}, {{0, 1, -5}, {0, 0, 1}}, {{0, 1.5, -2}, {0, 0, 1}}})
            v.push_back((double)local(k1, k.o, normalized(k.d)).size());
        emit("cylinder.constrained_counts", v);
        Shape k2 = k1;
        k2.closed = true;
        v.clear();
        for (auto k : std::vector<Case>{{{0, 3, 0}, {0, -1, 0}}, {{0, 3, -2}, {0, -1, 2}}, {{0, 4, -2}, {0, -1, 1}},
                                        {{0, 0, -2}, {0, 1, 2}}, {{0, -1, -2}, {0, 1, 1}}})
            v.push_back((double)local(k2, k.o, normalized(k.d)).size());
        emit("cylinder.caps_counts", v);
        v.clear();
        for (V3 p : {V3{0, 1, 0}, V3{0.5, 1, 0}, V3{0, 1, 0.5}, V3{0, 2, 0}, V3{0.5, 2, 0}, V3{0, 2, 0.5}}) {
            auto n = vv(local_normal_at(k2, p));
            v.insert(v.end(), n.begin(), n.end());
        }
        emit("cylinder.cap_normals", v);
    }
    {
        Shape c;
        c.kind = S_CONE;
        struct Case { V3 o, d; };
        std::vector<double> v;
        for (auto k : std::vector<Case>{{{0, 0, -5}, {0, 0, 1}}, {{0, 0, -5}, {1, 1, 1}}, {{1, 1, -5}, {-0.5, -1, 1}}}) {
            auto t = ts(local(c, k.o, normalized(k.d)));
            v.push_back((double)t.size());
            v.insert(v.end(), t.begin(), t.end());
        }
        emit("cone.intersects", v);
        emit("cone.parallel_to_half", ts(local(c, {0, 0, -1}, normalized({0, 1, 1}))));
        Shape k = c;
        k.minimum = -0.5;
        k.maximum = 0.5;
        k.closed = true;
        v.clear();
        for (auto q : std::vector<Case>{{{0, 0, -5}, {0, 1, 0}}, {{0, 0, -0.25}, {0, 1, 1}}, {{0, 0, -0.25}, {0, 1, 0}}})
            v.push_back((double)local(k, q.o, normalized(q.d)).size());
        emit("cone.caps_counts", v);
        v.clear();
        for (V3 p : {V3{0, 0, 0}, V3{1, 1, 1}, V3{-1, -1, 0}}) {
            auto n = vv(local_normal_at(c, p));
            v.insert(v.end(), n.begin(), n.end());
        }
        emit("cone.normals", v);
    }
    {
        Shape t = make_triangle({0, 1, 0}, {-1, 0, 0}, {1, 0, 0});
        auto v = vv(t.e1), e2 = vv(t.e2), n = vv(t.tn);
        v.insert(v.end(), e2.begin(), e2.end());
        v.insert(v.end(), n.begin(), n.end());
        emit("triangle.creating", v);
        emit("triangle.normal", vv(local_normal_at(t, {0, 0.5, 0})));
        emit("triangle.misses_counts",
             {(double)local(t, {0, -1, -2}, {0, 1, 0}).size(), (double)local(t, {1, 1, -2}, {0, 0, 1}).size(),
              (double)local(t, {-1, 1, -2}, {0, 0, 1}).size(), (double)local(t, {0, -1, -2}, {0, 0, 1}).size()});
        emit("triangle.intersects", ts(local(t, {0, 0.5, -2}, {0, 0, 1})));
    }

    // -------------------------------------------------------------- patterns
    {
        Pattern st;
        st.kind = P_STRIPE;
        st.a = WHITE;
        st.b = BLACK;
        std::vector<double> v;
        for (V3 p : {V3{0, 0, 0}, V3{0.9, 0, 0}, V3{1, 0, 0}, V3{-0.1, 0, 0}, V3{-1, 0, 0}, V3{-1.1, 0, 0},
                     V3{0, 1, 0}, V3{0, 2, 0}, V3{0, 0, 1}, V3{0, 0, 2}})
            v.push_back(pattern_color_at(st, p).r);
        emit("stripe.color_at_red", v);
        Shape s;
        s.material.pattern = std::make_shared<Pattern>(st);
        s.material.ambient = 1.0;
        s.material.diffuse = 0.0;
        s.material.specular = 0.0;
        Light l{{0, 10, -10}, WHITE};
        auto c1 = cv(lighting(s.material, s, l, {0.9, 0, 0}, {0, 0, -1}, {0, 0, -1}, false));
        auto c2 = cv(lighting(s.material, s, l, {1.1, 0, 0}, {0, 0, -1}, {0, 0, -1}, false));
        c1.insert(c1.end(), c2.begin(), c2.end());
        emit("stripe.lighting_with_pattern", c1);
        Shape sc;
        sc.set_transformation(scaling(2, 2, 2));
        Pattern pt = st;
        pt.set_transformation(scaling(2, 2, 2));
        Pattern pt2 = st;
        pt2.set_transformation(translation(0.5, 0, 0));
        emit("stripe.transforms", {pattern_color_at_shape(st, sc, {1.5, 0, 0}).r,
                                   pattern_color_at_shape(pt, s, {1.5, 0, 0}).r,
                                   pattern_color_at_shape(pt2, sc, {2.5, 0, 0}).r});
    }
    {
        Pattern g;
        g.kind = P_GRADIENT;
        g.a = WHITE;
        g.b = BLACK;
        std::vector<double> v;
        for (double x : {0.0, 0.25, 0.5, 0.75, 1.0}) {
            auto c = cv(pattern_color_at(g, {x, 0, 0}));
            v.insert(v.end(), c.begin(), c.end());
        }
        emit("gradient.color_at", v);
        Pattern r;
        r.kind = P_RING;
        r.a = WHITE;
        r.b = BLACK;
        v.clear();
        for (V3 p : {V3{0, 0, 0}, V3{1, 0, 0}, V3{0, 0, 1}, V3{0.708, 0, 0.708}}) v.push_back(pattern_color_at(r, p).r);
        emit("ring.color_at_red", v);
        Pattern k;
        k.kind = P_CHECKER;
        k.a = WHITE;
        k.b = BLACK;
        v.clear();
        for (V3 p : {V3{0, 0, 0}, V3{0.99, 0, 0}, V3{1.01, 0, 0}, V3{0, 0.99, 0}, V3{0, 1.01, 0}, V3{0, 0, 0.99},
                     V3{0, 0, 1.01}})
            v.push_back(pattern_color_at(k, p).r);
        emit("checker.color_at_red", v);
    }
    {
        Pattern t;
        t.kind = P_TEST;
        Shape s;
        s.set_transformation(scaling(2, 2, 2));
        auto a = cv(pattern_color_at_shape(t, s, {2, 3, 4}));
        Pattern t2 = t;
        t2.set_transformation(scaling(2, 2, 2));
        Shape d;
        auto b = cv(pattern_color_at_shape(t2, d, {2, 3, 4}));
        Pattern t3 = t;
        t3.set_transformation(translation(0.5, 1, 1.5));
        auto c = cv(pattern_color_at_shape(t3, s, {2.5, 3, 3.5}));
        a.insert(a.end(), b.begin(), b.end());
        a.insert(a.end(), c.begin(), c.end());
        emit("pattern.test_pattern_transforms", a);
    }

    // --------------------------------------------------- matrix / transforms
    {
        M4 a{{{1, 2, 3, 4}, {5, 6, 7, 8}, {9, 8, 7, 6}, {5, 4, 3, 2}}};
        M4 b{{{-2, 1, 2, 3}, {3, 2, 1, -1}, {4, 3, 6, 5}, {1, 2, 7, 8}}};
        emit("matrix.multiply", mv(mul(a, b)));
        M4 c{{{1, 2, 3, 4}, {2, 4, 4, 2}, {8, 6, 4, 1}, {0, 0, 0, 1}}};
        emit("matrix.multiply_point", vv(mul_point(c, {1, 2, 3})));
        M2 d2{{{1, 5}, {-3, 2}}};
        M3 d3{{{1, 2, 6}, {-5, 8, -4}, {2, 6, 4}}};
        M4 d4{{{-2, -8, 3, 5}, {-3, 1, 7, 3}, {1, 2, -9, 6}, {-6, 7, 7, -9}}};
        emit("matrix.determinants", {determinant(d2), cofactor(d3, 0, 0), cofactor(d3, 0, 1), cofactor(d3, 0, 2),
                                     determinant(d3), cofactor(d4, 0, 0), cofactor(d4, 0, 1), cofactor(d4, 0, 2),
                                     cofactor(d4, 0, 3), determinant(d4)});
        M3 m3{{{3, 5, 0}, {2, -1, -7}, {6, -1, 5}}};
        emit("matrix.minor_cofactor", {minor3(m3, 0, 0), cofactor(m3, 0, 0), minor3(m3, 1, 0), cofactor(m3, 1, 0)});
        M4 i1{{{-5, 2, 6, -8}, {1, -5, 1, 8}, {7, 7, -6, -7}, {1, -3, 7, 4}}};
        M4 i3{{{9, 3, 0, 9}, {-5, -2, 6, -3}, {-4, 9, 6, 4}, {-7, 6, 6, 2}}};
        emit("matrix.inverse_1", mv(inverse(i1)));
        emit("matrix.inverse_1_terms", {determinant(i1), cofactor(i1, 2, 3), cofactor(i1, 3, 2)});
        emit("matrix.inverse_3", mv(inverse(i3)));
    }
    {
        emit("transform.view_default", mv(view_transform({0, 0, 0}, {0, 0, -1}, {0, 1, 0})));
        emit("transform.view_positive_z", mv(view_transform({0, 0, 0}, {0, 0, 1}, {0, 1, 0})));
        emit("transform.view_moves_world", mv(view_transform({0, 0, 8}, {0, 0, 0}, {0, 1, 0})));
        emit("transform.view_complex", mv(view_transform({1, 3, 2}, {4, -2, 8}, {1, 1, 0})));
        std::vector<double> v;
        const M4 sh[6] = {shearing(1, 0, 0, 0, 0, 0), shearing(0, 1, 0, 0, 0, 0), shearing(0, 0, 1, 0, 0, 0),
                          shearing(0, 0, 0, 1, 0, 0), shearing(0, 0, 0, 0, 1, 0), shearing(0, 0, 0, 0, 0, 1)};
        for (const M4& m : sh) {
            auto p = vv(mul_point(m, {2, 3, 4}));
            v.insert(v.end(), p.begin(), p.end());
        }
        emit("transform.shearing", v);
        M4 tot = mul(mul(translation(10, 5, 7), scaling(5, 5, 5)), rotation_x(PI / 2.0));
        emit("transform.chained", vv(mul_point(tot, {1, 0, 1})));
    }
    std::printf("\n}\n");
    return 0;
}
