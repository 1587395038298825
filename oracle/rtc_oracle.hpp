// rtc_oracle.hpp — CPU f64 restatement of przemo199/ray-tracer-challenge-rs's
// render path.  TEST INFRASTRUCTURE ONLY: this is the parity checker and the
// CPU baseline ("kind": "port") of bench.py.  Nothing in the product
// (ray-tracer-challenge-rs_amd/) includes, links or calls it.
//
// Restated from the reference, file by file (paths under /root/reference):
//   consts.rs, utils.rs, primitives/{vector,point,color,light,matrix,
//   transformations}.rs, shapes/*.rs, patterns/*.rs,
//   composites/{ray,intersection,intersections,computed_hit,material,world,
//   camera,canvas}.rs
// Same operation order, the same explicit FMA at every `mul_add` site, no
// contraction elsewhere (build with -ffp-contract=off, no -ffast-math), a
// stable sort of intersections, value equality for shape identity.
// Pinned against the reference's own unit-test known answers
// (tests/golden/reference_kats.json, tests/test_oracle_kat.py).
#pragma once

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <memory>
#include <thread>
#include <vector>

namespace orc {

// consts.rs:2-8
constexpr double EPSILON = 0.00000008;
constexpr double MINV = -DBL_MAX;
constexpr double MAXV = DBL_MAX;
constexpr double PI = 3.14159265358979323846264338327950288;

// utils.rs:16-24
inline bool coarse_eq(double a, double b) {
    if (a == b) return true;
    return std::fabs(a - b) < EPSILON;
}
inline double sq(double v) { return v * v; }  // utils.rs Squared

// f64 `as i64` is saturating, NaN -> 0 (Rust semantics)
inline int64_t sat_i64(double v) {
    if (std::isnan(v)) return 0;
    if (v >= 9223372036854775807.0) return INT64_MAX;
    if (v <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)v;
}

// utils.rs:47-57
inline bool solve_quadratic(double a, double b, double c, double& s1, double& s2) {
    double disc = std::fma(4.0 * a, -c, sq(b));
    if (disc < 0.0) return false;
    double double_a = 2.0 * a;
    double root = std::sqrt(disc);
    s1 = (-b - root) / double_a;
    s2 = (-b + root) / double_a;
    return true;
}

// ---------------------------------------------------------------- primitives
// vector.rs / point.rs: three f64 components, w implied by the type.
struct V3 {
    double x = 0, y = 0, z = 0;
    V3() = default;
    V3(double a, double b, double c) : x(a), y(b), z(c) {}
    double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
using Point = V3;
using Vector = V3;

inline V3 add(const V3& a, const V3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(const V3& a, const V3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 scale(const V3& a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 neg(const V3& a) { return {-a.x, -a.y, -a.z}; }
// vector.rs:84-86
inline double magnitude(const V3& v) { return std::sqrt(sq(v.x) + sq(v.y) + sq(v.z)); }
// vector.rs:88-91
inline V3 normalized(const V3& v) {
    double m = magnitude(v);
    return {v.x / m, v.y / m, v.z / m};
}
// vector.rs:93-95
inline double dot(const V3& a, const V3& b) { return std::fma(a.z, b.z, std::fma(a.x, b.x, a.y * b.y)); }
// vector.rs:97-103
inline V3 cross(const V3& a, const V3& b) {
    return {std::fma(a.y, b.z, -a.z * b.y), std::fma(a.z, b.x, -a.x * b.z), std::fma(a.x, b.y, -a.y * b.x)};
}
// vector.rs:105-107: self - (normal * 2.0 * self.dot(normal))
inline V3 reflect(const V3& v, const V3& n) {
    double d = dot(v, n);
    return sub(v, scale(scale(n, 2.0), d));
}
inline bool coarse_eq(const V3& a, const V3& b) {
    return coarse_eq(a.x, b.x) && coarse_eq(a.y, b.y) && coarse_eq(a.z, b.z);
}

// color.rs
struct Color {
    double r = 0, g = 0, b = 0;
    Color() = default;
    Color(double a, double c, double d) : r(a), g(c), b(d) {}
};
inline Color cadd(const Color& a, const Color& b) { return {a.r + b.r, a.g + b.g, a.b + b.b}; }
inline Color csub(const Color& a, const Color& b) { return {a.r - b.r, a.g - b.g, a.b - b.b}; }
inline Color cmul(const Color& a, const Color& b) { return {a.r * b.r, a.g * b.g, a.b * b.b}; }
inline Color cscale(const Color& a, double s) { return {a.r * s, a.g * s, a.b * s}; }
inline bool coarse_eq(const Color& a, const Color& b) {
    return coarse_eq(a.r, b.r) && coarse_eq(a.g, b.g) && coarse_eq(a.b, b.b);
}
const Color BLACK{0, 0, 0};
const Color WHITE{1, 1, 1};

// light.rs:6-10
struct Light {
    Point position;
    Color intensity;
};

// ------------------------------------------------------------------- matrix
// matrix.rs: const-generic square matrices, row-major [[f64;N];N].
template <int N>
struct Mat {
    double m[N][N];
    static Mat null() {
        Mat r;
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) r.m[i][j] = 0.0;
        return r;
    }
    static Mat identity() {
        Mat r = null();
        for (int i = 0; i < N; ++i) r.m[i][i] = 1.0;
        return r;
    }
    bool operator==(const Mat& o) const {
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j)
                if (!(m[i][j] == o.m[i][j])) return false;
        return true;
    }
};
using M2 = Mat<2>;
using M3 = Mat<3>;
using M4 = Mat<4>;

// matrix.rs:30-43
template <int N>
Mat<N> transpose(const Mat<N>& a) {
    Mat<N> r;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) r.m[i][j] = a.m[j][i];
    return r;
}
// matrix.rs:45-51
template <int N>
bool is_identity(const Mat<N>& a) {
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j)
            if (!coarse_eq(a.m[i][j], i == j ? 1.0 : 0.0)) return false;
    return true;
}
template <int N>
bool coarse_eq(const Mat<N>& a, const Mat<N>& b) {
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j)
            if (!coarse_eq(a.m[i][j], b.m[i][j])) return false;
    return true;
}
// matrix.rs:317-330: left-to-right fold from 0.0, no FMA
template <int N>
Mat<N> mul(const Mat<N>& a, const Mat<N>& b) {
    Mat<N> r;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            double acc = 0.0;
            for (int k = 0; k < N; ++k) acc = acc + (a.m[i][k] * b.m[k][j]);
            r.m[i][j] = acc;
        }
    return r;
}
// matrix.rs:332-346 (Point, w = 1) and 348-362 (Vector, w = 0)
inline Point mul_point(const M4& a, const Point& p) {
    double v[4] = {p.x, p.y, p.z, 1.0};
    double o[3];
    for (int r = 0; r < 3; ++r) {
        double acc = 0.0;
        for (int c = 0; c < 4; ++c) acc = acc + (a.m[r][c] * v[c]);
        o[r] = acc;
    }
    return {o[0], o[1], o[2]};
}
inline Vector mul_vector(const M4& a, const Vector& p) {
    double v[4] = {p.x, p.y, p.z, 0.0};
    double o[3];
    for (int r = 0; r < 3; ++r) {
        double acc = 0.0;
        for (int c = 0; c < 4; ++c) acc = acc + (a.m[r][c] * v[c]);
        o[r] = acc;
    }
    return {o[0], o[1], o[2]};
}

// matrix.rs:65-119
inline double determinant(const M2& a) { return (a.m[0][0] * a.m[1][1]) - (a.m[0][1] * a.m[1][0]); }
inline double minor2(const M2& a, int row, int col) {
    // Matrix<2>::submatrix returns the single remaining element
    for (int r = 0; r < 2; ++r) {
        if (r == row) continue;
        for (int c = 0; c < 2; ++c) {
            if (c == col) continue;
            return a.m[r][c];
        }
    }
    return 0.0;
}
inline double cofactor(const M2& a, int row, int col) {
    double mi = minor2(a, row, col);
    return ((row + col) % 2 == 0) ? mi : -mi;
}
inline M2 inverse(const M2& a) {
    if (is_identity(a)) return M2::identity();
    M2 r = M2::null();
    double det = determinant(a);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) r.m[i][j] = cofactor(a, j, i) / det;
    return r;
}
// matrix.rs:121-187
inline M2 submatrix(const M3& a, int er, int ec) {
    M2 r = M2::null();
    for (int i = 0; i < 3; ++i) {
        if (i == er) continue;
        for (int j = 0; j < 3; ++j) {
            if (j == ec) continue;
            r.m[i < er ? i : i - 1][j < ec ? j : j - 1] = a.m[i][j];
        }
    }
    return r;
}
inline double cofactor(const M3& a, int row, int col);
inline double determinant(const M3& a) {
    double acc = 0.0;
    for (int i = 0; i < 3; ++i) acc = acc + (a.m[0][i] * cofactor(a, 0, i));
    return acc;
}
inline double minor3(const M3& a, int row, int col) { return determinant(submatrix(a, row, col)); }
inline double cofactor(const M3& a, int row, int col) {
    double mi = minor3(a, row, col);
    return ((row + col) % 2 == 0) ? mi : -mi;
}
inline M3 inverse(const M3& a) {
    if (is_identity(a)) return M3::identity();
    M3 r = M3::null();
    double det = determinant(a);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = cofactor(a, j, i) / det;
    return r;
}
// matrix.rs:189-259 (note the is_identity shortcut inside submatrix, 192-194)
inline M3 submatrix(const M4& a, int er, int ec) {
    if (is_identity(a)) return M3::identity();
    M3 r = M3::null();
    for (int i = 0; i < 4; ++i) {
        if (i == er) continue;
        for (int j = 0; j < 4; ++j) {
            if (j == ec) continue;
            r.m[i < er ? i : i - 1][j < ec ? j : j - 1] = a.m[i][j];
        }
    }
    return r;
}
inline double cofactor(const M4& a, int row, int col) {
    double mi = determinant(submatrix(a, row, col));
    return ((row + col) % 2 == 0) ? mi : -mi;
}
inline double determinant(const M4& a) {
    double acc = 0.0;
    for (int i = 0; i < 4; ++i) acc = acc + (a.m[0][i] * cofactor(a, 0, i));
    return acc;
}
inline M4 inverse(const M4& a) {
    if (is_identity(a)) return M4::identity();
    M4 r = M4::null();
    double det = determinant(a);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.m[i][j] = cofactor(a, j, i) / det;
    return r;
}

// transformations.rs:5-87
inline M4 translation(double x, double y, double z) {
    M4 r = M4::identity();
    r.m[0][3] = x;
    r.m[1][3] = y;
    r.m[2][3] = z;
    return r;
}
inline M4 scaling(double x, double y, double z) {
    M4 r = M4::identity();
    r.m[0][0] = x;
    r.m[1][1] = y;
    r.m[2][2] = z;
    return r;
}
inline M4 rotation_x(double t) {
    M4 r = M4::identity();
    double c = std::cos(t), s = std::sin(t);
    r.m[1][1] = c;
    r.m[1][2] = -s;
    r.m[2][1] = s;
    r.m[2][2] = c;
    return r;
}
inline M4 rotation_y(double t) {
    M4 r = M4::identity();
    double c = std::cos(t), s = std::sin(t);
    r.m[0][0] = c;
    r.m[0][2] = s;
    r.m[2][0] = -s;
    r.m[2][2] = c;
    return r;
}
inline M4 rotation_z(double t) {
    M4 r = M4::identity();
    double c = std::cos(t), s = std::sin(t);
    r.m[0][0] = c;
    r.m[0][1] = -s;
    r.m[1][0] = s;
    r.m[1][1] = c;
    return r;
}
inline M4 shearing(double xy, double xz, double yx, double yz, double zx, double zy) {
    M4 r = M4::identity();
    r.m[0][1] = xy;
    r.m[0][2] = xz;
    r.m[1][0] = yx;
    r.m[1][2] = yz;
    r.m[2][0] = zx;
    r.m[2][1] = zy;
    return r;
}
inline M4 view_transform(const Point& from, const Point& to, const Vector& up) {
    Vector forward = normalized(sub(to, from));
    Vector upn = normalized(up);
    Vector left = cross(forward, upn);
    Vector true_up = cross(left, forward);
    M4 o = M4::null();
    o.m[0][0] = left.x; o.m[0][1] = left.y; o.m[0][2] = left.z; o.m[0][3] = 0.0;
    o.m[1][0] = true_up.x; o.m[1][1] = true_up.y; o.m[1][2] = true_up.z; o.m[1][3] = 0.0;
    o.m[2][0] = -forward.x; o.m[2][1] = -forward.y; o.m[2][2] = -forward.z; o.m[2][3] = 0.0;
    o.m[3][0] = 0.0; o.m[3][1] = 0.0; o.m[3][2] = 0.0; o.m[3][3] = 1.0;
    return mul(o, translation(-from.x, -from.y, -from.z));
}

// --------------------------------------------------------------------- ray
// ray.rs
struct Ray {
    Point origin;
    Vector direction;
};
inline Point position(const Ray& r, double t) { return add(r.origin, scale(r.direction, t)); }
inline Ray transform(const Ray& r, const M4& m) { return {mul_point(m, r.origin), mul_vector(m, r.direction)}; }

// ----------------------------------------------------------------- patterns
// patterns/*.rs
enum PatternKind { P_STRIPE = 0, P_GRADIENT = 1, P_RING = 2, P_CHECKER = 3, P_COMPLEX = 4, P_TEST = 5 };
struct Pattern {
    int kind = P_STRIPE;
    Color a, b;
    M4 inv = M4::identity();
    std::shared_ptr<Pattern> sub_a, sub_b;
    void set_transformation(const M4& t) { inv = inverse(t); }
};
using PatternPtr = std::shared_ptr<Pattern>;

inline bool pattern_eq(const Pattern* p, const Pattern* q);
inline Color pattern_color_at(const Pattern& p, const Point& pt) {
    switch (p.kind) {
        case P_STRIPE: {  // stripe_pattern.rs:24-31
            int64_t d = sat_i64(std::floor(pt.x));
            return (d % 2 == 0) ? p.a : p.b;
        }
        case P_GRADIENT: {  // gradient_pattern.rs:24-31
            Color dist = csub(p.b, p.a);
            double fraction = std::fabs(pt.x - std::trunc(pt.x));
            if (sat_i64(pt.x) % 2 != 0) fraction = 1.0 - fraction;
            return cadd(p.a, cscale(dist, fraction));
        }
        case P_RING: {  // ring_pattern.rs:25-32
            int64_t d = sat_i64(std::floor(std::sqrt(sq(pt.x) + sq(pt.z))));
            return (d % 2 == 0) ? p.a : p.b;
        }
        case P_CHECKER: {  // checker_pattern.rs:24-31
            int64_t d = sat_i64(std::floor(pt.x) + std::floor(pt.y) + std::floor(pt.z));
            return (d % 2 == 0) ? p.a : p.b;
        }
        case P_COMPLEX: {  // complex_pattern.rs:25-32 (sub-pattern transforms ignored)
            int64_t d = sat_i64(std::floor(pt.x));
            return (d % 2 == 0) ? pattern_color_at(*p.sub_a, pt) : pattern_color_at(*p.sub_b, pt);
        }
        default:  // TestPattern, pattern.rs:55-58
            return {pt.x, pt.y, pt.z};
    }
}

// ----------------------------------------------------------------- material
// material.rs:8-20, Default 157-161
struct Material {
    Color color = WHITE;
    PatternPtr pattern;
    double ambient = 0.1, diffuse = 0.9, specular = 0.9, shininess = 200.0;
    double reflectiveness = 0.0, refractive_index = 1.0, transparency = 0.0;
    bool casts_shadow = true;
    static Material glass() {  // material.rs:148-154
        Material m;
        m.transparency = 1.0;
        m.refractive_index = 1.5;
        return m;
    }
};
constexpr double DEFAULT_REFRACTIVE_INDEX = 1.0;  // material.rs:24

inline bool pattern_eq(const Pattern* p, const Pattern* q) {
    if (p == q) return true;
    if (!p || !q) return false;
    if (p->kind != q->kind) return false;
    if (p->kind == P_COMPLEX) return pattern_eq(p->sub_a.get(), q->sub_a.get()) && pattern_eq(p->sub_b.get(), q->sub_b.get()) && p->inv == q->inv;
    if (p->kind == P_TEST) return p->inv == q->inv;
    return p->a.r == q->a.r && p->a.g == q->a.g && p->a.b == q->a.b && p->b.r == q->b.r && p->b.g == q->b.g &&
           p->b.b == q->b.b && p->inv == q->inv;
}
inline bool material_eq(const Material& a, const Material& b) {  // #[derive(PartialEq)]
    return a.color.r == b.color.r && a.color.g == b.color.g && a.color.b == b.color.b &&
           pattern_eq(a.pattern.get(), b.pattern.get()) && a.ambient == b.ambient && a.diffuse == b.diffuse &&
           a.specular == b.specular && a.shininess == b.shininess && a.reflectiveness == b.reflectiveness &&
           a.refractive_index == b.refractive_index && a.transparency == b.transparency &&
           a.casts_shadow == b.casts_shadow;
}

// ------------------------------------------------------------------- shapes
enum ShapeKind { S_SPHERE = 0, S_PLANE = 1, S_CUBE = 2, S_CYLINDER = 3, S_CONE = 4, S_TRIANGLE = 5 };
struct Shape {
    int kind = S_SPHERE;
    Material material;
    M4 inv = M4::identity();
    double minimum = MINV, maximum = MAXV;  // cylinder/cone Default (cylinder.rs:133-141)
    bool closed = false;
    Point v1, v2, v3;  // triangle.rs:12-17
    Vector e1, e2, tn;
    void set_transformation(const M4& t) { inv = inverse(t); }
};
inline Shape make_triangle(const Point& p1, const Point& p2, const Point& p3) {  // triangle.rs:21-35
    Shape s;
    s.kind = S_TRIANGLE;
    s.v1 = p1; s.v2 = p2; s.v3 = p3;
    s.e1 = sub(p2, p1);
    s.e2 = sub(p3, p1);
    s.tn = normalized(cross(s.e2, s.e1));
    return s;
}
// dyn Shape PartialEq (shape.rs:34-38 → dyn_partial_eq.rs:14-16 → derive)
inline bool shape_eq(const Shape& a, const Shape& b) {
    if (&a == &b) return true;
    if (a.kind != b.kind) return false;
    if (!material_eq(a.material, b.material) || !(a.inv == b.inv)) return false;
    if (a.kind == S_CYLINDER || a.kind == S_CONE)
        return a.minimum == b.minimum && a.maximum == b.maximum && a.closed == b.closed;
    if (a.kind == S_TRIANGLE) {
        auto eq = [](const V3& u, const V3& v) { return u.x == v.x && u.y == v.y && u.z == v.z; };
        return eq(a.v1, b.v1) && eq(a.v2, b.v2) && eq(a.v3, b.v3) && eq(a.e1, b.e1) && eq(a.e2, b.e2) && eq(a.tn, b.tn);
    }
    return true;
}

// intersection.rs:7-11
struct Hit {
    double t;
    const Shape* shape;
};
using Hits = std::vector<Hit>;

// cube.rs:22-43
inline void cube_check_axis(double origin, double direction, double& tmin, double& tmax) {
    double nmin = -1.0 - origin;
    double nmax = 1.0 - origin;
    if (std::fabs(direction) >= EPSILON) {
        tmin = nmin / direction;
        tmax = nmax / direction;
    } else {
        tmin = nmin * MAXV;
        tmax = nmax * MAXV;
    }
    if (tmin > tmax) std::swap(tmin, tmax);
}
// Rust f64::max / f64::min ignore a NaN operand (IEEE maxNum/minNum).
inline double rmax(double a, double b) { return std::fmax(a, b); }
inline double rmin(double a, double b) { return std::fmin(a, b); }

// cylinder.rs:34-39 / cone.rs:34-39
inline bool check_cap(const Ray& r, double t, double radius) {
    double x = std::fma(r.direction.x, t, r.origin.x);
    double z = std::fma(r.direction.z, t, r.origin.z);
    return (sq(x) + sq(z)) <= sq(radius);
}

inline void local_intersect(const Shape& s, const Ray& r, Hits& out) {
    switch (s.kind) {
        case S_SPHERE: {  // sphere.rs:41-53
            Vector o = r.origin;
            double a = dot(r.direction, r.direction);
            double b = 2.0 * dot(r.direction, o);
            double c = dot(o, o) - 1.0;
            double t1, t2;
            if (solve_quadratic(a, b, c, t1, t2)) {
                out.push_back({t1, &s});
                out.push_back({t2, &s});
            }
            return;
        }
        case S_PLANE: {  // plane.rs:42-48
            if (std::fabs(r.direction.y) < EPSILON) return;
            out.push_back({-r.origin.y / r.direction.y, &s});
            return;
        }
        case S_CUBE: {  // cube.rs:65-85
            double xn, xx, yn, yx, zn, zx;
            cube_check_axis(r.origin.x, r.direction.x, xn, xx);
            cube_check_axis(r.origin.y, r.direction.y, yn, yx);
            cube_check_axis(r.origin.z, r.direction.z, zn, zx);
            double tmin = rmax(rmax(rmax(MINV, xn), yn), zn);
            double tmax = rmin(rmin(rmin(MAXV, xx), yx), zx);
            if (tmin < tmax && tmax > 0.0) {
                out.push_back({tmin, &s});
                out.push_back({tmax, &s});
            }
            return;
        }
        case S_CYLINDER: {  // cylinder.rs:81-110
            double a = sq(r.direction.x) + sq(r.direction.z);
            if (std::fabs(a) > 0.0) {
                double b = 2.0 * std::fma(r.origin.x, r.direction.x, r.origin.z * r.direction.z);
                double c = sq(r.origin.x) + sq(r.origin.z) - 1.0;
                double t1, t2;
                if (solve_quadratic(a, b, c, t1, t2)) {
                    if (t1 > t2) std::swap(t1, t2);
                    double y1 = std::fma(t1, r.direction.y, r.origin.y);
                    if (s.minimum < y1 && y1 < s.maximum) out.push_back({t1, &s});
                    double y2 = std::fma(t2, r.direction.y, r.origin.y);
                    if (s.minimum < y2 && y2 < s.maximum) out.push_back({t2, &s});
                }
            }
            // cylinder.rs:41-58 intersect_caps
            if (!s.closed || std::fabs(r.direction.y) < EPSILON) return;
            double t = (s.minimum - r.origin.y) / r.direction.y;
            if (check_cap(r, t, 1.0)) out.push_back({t, &s});
            t = (s.maximum - r.origin.y) / r.direction.y;
            if (check_cap(r, t, 1.0)) out.push_back({t, &s});
            return;
        }
        case S_CONE: {  // cone.rs:81-112
            double a = sq(r.direction.x) - sq(r.direction.y) + sq(r.direction.z);
            double b = 2.0 * std::fma(r.origin.z, r.direction.z,
                                      std::fma(r.origin.x, r.direction.x, -r.origin.y * r.direction.y));
            double c = sq(r.origin.x) - sq(r.origin.y) + sq(r.origin.z);
            double t1, t2;
            if (std::fabs(a) < EPSILON && std::fabs(b) > EPSILON) {
                out.push_back({-c / (2.0 * b), &s});
            } else if (solve_quadratic(a, b, c, t1, t2)) {
                if (t1 > t2) std::swap(t1, t2);
                double y1 = std::fma(r.direction.y, t1, r.origin.y);
                if (s.minimum < y1 && y1 < s.maximum) out.push_back({t1, &s});
                double y2 = std::fma(r.direction.y, t2, r.origin.y);
                if (s.minimum < y2 && y2 < s.maximum) out.push_back({t2, &s});
            }
            // cone.rs:41-58 intersect_caps (radius = |min|, |max| via squared)
            if (!s.closed || std::fabs(r.direction.y) < EPSILON) return;
            double t = (s.minimum - r.origin.y) / r.direction.y;
            if (check_cap(r, t, s.minimum)) out.push_back({t, &s});
            t = (s.maximum - r.origin.y) / r.direction.y;
            if (check_cap(r, t, s.maximum)) out.push_back({t, &s});
            return;
        }
        default: {  // triangle.rs:39-56
            Vector dce2 = cross(r.direction, s.e2);
            double det = dot(s.e1, dce2);
            if (std::fabs(det) < EPSILON) return;
            Vector v1o = sub(r.origin, s.v1);
            double u = dot(v1o, dce2) / det;
            if (!(u >= 0.0 && u <= 1.0)) return;
            Vector oce1 = cross(v1o, s.e1);
            double v = dot(r.direction, oce1) / det;
            if (v > 0.0 && u + v < 1.0) out.push_back({dot(s.e2, oce1) / det, &s});
            return;
        }
    }
}

inline Vector local_normal_at(const Shape& s, const Point& p) {
    switch (s.kind) {
        case S_SPHERE: return {p.x, p.y, p.z};  // sphere.rs:57-59
        case S_PLANE: return {0.0, 1.0, 0.0};   // plane.rs:52-54
        case S_CUBE: {                          // cube.rs:89-101
            V3 ap{std::fabs(p.x), std::fabs(p.y), std::fabs(p.z)};
            double mx = rmax(rmax(rmax(MINV, ap.x), ap.y), ap.z);
            if (coarse_eq(mx, ap.x)) return {p.x, 0.0, 0.0};
            if (coarse_eq(mx, ap.y)) return {0.0, p.y, 0.0};
            return {0.0, 0.0, p.z};
        }
        case S_CYLINDER: {  // cylinder.rs:114-126
            double d = sq(p.x) + sq(p.z);
            if (d < 1.0 && p.y >= (s.maximum - EPSILON)) return {0.0, 1.0, 0.0};
            if (d < 1.0 && p.y <= (s.minimum + EPSILON)) return {0.0, -1.0, 0.0};
            return {p.x, 0.0, p.z};
        }
        case S_CONE: {  // cone.rs:116-133
            double d = sq(p.x) + sq(p.z);
            if (d < sq(s.maximum) && p.y >= (s.maximum - EPSILON)) return {0.0, 1.0, 0.0};
            if (d < sq(s.minimum) && p.y <= (s.minimum + EPSILON)) return {0.0, -1.0, 0.0};
            double y = std::sqrt(d);
            if (p.y > 0.0) y = -y;
            return {p.x, y, p.z};
        }
        default: return s.tn;  // triangle.rs:78-80
    }
}

// shape.rs:22-27
inline Vector normal_at(const Shape& s, const Point& p) {
    Point lp = mul_point(s.inv, p);
    Vector ln = local_normal_at(s, lp);
    Vector wn = mul_vector(transpose(s.inv), ln);
    return normalized(wn);
}

// pattern.rs:10-14
inline Color pattern_color_at_shape(const Pattern& p, const Shape& s, const Point& pt) {
    Point op = mul_point(s.inv, pt);
    Point pp = mul_point(p.inv, op);
    return pattern_color_at(p, pp);
}

// material.rs:53-114
inline Color lighting(const Material& m, const Shape& s, const Light& l, const Point& pt, const Vector& eye,
                      const Vector& normal, bool in_shadow) {
    Color resolved = m.pattern ? pattern_color_at_shape(*m.pattern, s, pt) : m.color;
    Color eff = cmul(resolved, l.intensity);
    Color ambient = cscale(eff, m.ambient);
    if (in_shadow) return ambient;
    Vector ld = normalized(sub(l.position, pt));
    double ldn = dot(ld, normal);
    if (ldn < 0.0) return ambient;
    Color diffuse = cscale(cscale(eff, m.diffuse), ldn);
    Vector rd = reflect(neg(ld), normal);
    double rde = dot(rd, eye);
    if (rde <= 0.0) return cadd(ambient, diffuse);
    double factor = std::pow(rde, m.shininess);
    Color specular = cscale(cscale(l.intensity, m.specular), factor);
    return cadd(cadd(ambient, diffuse), specular);
}

// computed_hit.rs:6-19
struct Comps {
    double t = 0;
    const Shape* shape = nullptr;
    Point point, over_point, under_point;
    Vector eye, normal, reflectv;
    double n1 = 1.0, n2 = 1.0;
    bool inside = false;
};

// intersection.rs:21-75
inline Comps prepare_computations(const Hit& hit, const Ray& ray, const Hits& xs) {
    Comps c;
    c.t = hit.t;
    c.shape = hit.shape;
    c.point = position(ray, hit.t);
    c.normal = normal_at(*hit.shape, c.point);
    c.eye = neg(ray.direction);
    c.inside = dot(c.normal, c.eye) < 0.0;
    if (c.inside) c.normal = neg(c.normal);
    c.reflectv = reflect(ray.direction, c.normal);
    std::vector<const Shape*> containers;
    for (const Hit& x : xs) {
        bool is_self = (hit.t == x.t) && shape_eq(*hit.shape, *x.shape);
        if (is_self) c.n1 = containers.empty() ? DEFAULT_REFRACTIVE_INDEX : containers.back()->material.refractive_index;
        auto it = std::find_if(containers.begin(), containers.end(),
                               [&](const Shape* q) { return shape_eq(*q, *x.shape); });
        if (it != containers.end())
            containers.erase(it);
        else
            containers.push_back(x.shape);
        if (is_self) {
            c.n2 = containers.empty() ? DEFAULT_REFRACTIVE_INDEX : containers.back()->material.refractive_index;
            break;
        }
    }
    // computed_hit.rs:33-34
    c.over_point = add(c.point, scale(c.normal, EPSILON));
    c.under_point = sub(c.point, scale(c.normal, EPSILON));
    return c;
}

// computed_hit.rs:50-68
inline double schlick(const Comps& c) {
    double cs = dot(c.eye, c.normal);
    if (c.n1 > c.n2) {
        double ratio = c.n1 / c.n2;
        double sin2_t = sq(ratio) * (1.0 - sq(cs));
        if (sin2_t > 1.0) return 1.0;
        cs = std::sqrt(1.0 - sin2_t);
    }
    double r0 = sq((c.n1 - c.n2) / (c.n1 + c.n2));
    double x = 1.0 - cs;
    double p5 = x * ((x * x) * (x * x));  // powi(5): LLVM's square-and-multiply expansion
    return std::fma(1.0 - r0, p5, r0);
}

// Counters in the reference's ray semantics.
// Per generation, indexed by `remaining` (world.rs:70-86; a child runs at
// its parent's remaining - 1): radiance rays traced (internal_color_at
// calls) and hits shaded.  Depths above kMaxRemaining are not counted.
struct Counters {
    static constexpr int kMaxRemaining = 16;  // rtc.h RT_MAX_SUPPORTED_DEPTH
    uint64_t primary = 0, shadow = 0, reflect = 0, refract = 0, shaded = 0;
    uint64_t lit_patterned = 0, refract_evals = 0, schlick_evals = 0;
    uint64_t traced_at[kMaxRemaining + 1] = {}, shaded_at[kMaxRemaining + 1] = {};
    void merge(const Counters& o) {
        primary += o.primary; shadow += o.shadow; reflect += o.reflect; refract += o.refract;
        shaded += o.shaded; lit_patterned += o.lit_patterned; refract_evals += o.refract_evals;
        schlick_evals += o.schlick_evals;
        for (int i = 0; i <= kMaxRemaining; ++i) {
            traced_at[i] += o.traced_at[i];
            shaded_at[i] += o.shaded_at[i];
        }
    }
};

// -------------------------------------------------------------------- world
struct World {
    std::vector<Light> lights;
    std::vector<Shape> shapes;  // world order; stable addresses once built
    static constexpr int MAX_REFLECTION_ITERATIONS = 6;  // world.rs:15

    // world.rs:25-35
    void collect_intersections(const Ray& r, Hits& xs) const {
        xs.clear();
        for (const Shape& s : shapes) local_intersect(s, transform(r, s.inv), xs);
        std::stable_sort(xs.begin(), xs.end(), [](const Hit& a, const Hit& b) { return a.t < b.t; });
    }
    // intersections.rs:13-18: first minimum of the t >= 0 entries
    static const Hit* hit(const Hits& xs) {
        const Hit* best = nullptr;
        for (const Hit& x : xs)
            if (x.t >= 0.0 && (!best || x.t < best->t)) best = &x;
        return best;
    }
    // world.rs:98-112
    bool is_in_shadow(const Light& l, const Point& p, Hits& xs) const {
        Vector v = sub(l.position, p);
        double dist = magnitude(v);
        Ray sr{p, normalized(v)};
        collect_intersections(sr, xs);
        for (const Hit& x : xs)
            if (x.shape->material.casts_shadow && x.t >= 0.0 && x.t < dist) return true;
        return false;
    }
    // world.rs:38-67
    Color shade_hit(const Comps& c, Hits& xs, int remaining, Counters* k = nullptr) const {
        const Material& m = c.shape->material;
        Color surface = BLACK;
        for (const Light& l : lights) {
            bool shadowed = is_in_shadow(l, c.over_point, xs);
            if (k) {
                k->shadow++;
                if (m.pattern) k->lit_patterned++;
            }
            surface = cadd(surface, lighting(m, *c.shape, l, c.over_point, c.eye, c.normal, shadowed));
        }
        Color refl = reflected_color(c, xs, remaining, k);
        Color refr = refracted_color(c, xs, remaining, k);
        if (m.reflectiveness > 0.0 && m.transparency > 0.0) {
            if (k) k->schlick_evals++;
            double r = schlick(c);
            return cadd(cadd(surface, cscale(refl, r)), cscale(refr, 1.0 - r));
        }
        return cadd(cadd(surface, refl), refr);
    }
    // world.rs:70-86
    Color internal_color_at(const Ray& r, Hits& xs, int remaining, Counters* k = nullptr) const {
        const bool counted = k && remaining >= 0 && remaining <= Counters::kMaxRemaining;
        if (counted) k->traced_at[remaining]++;
        collect_intersections(r, xs);
        Hits shading;
        const Hit* h = hit(xs);
        if (!h) return BLACK;
        if (k) k->shaded++;
        if (counted) k->shaded_at[remaining]++;
        Comps c = prepare_computations(*h, r, xs);
        return shade_hit(c, shading, remaining, k);
    }
    // world.rs:89-95
    Color color_at(const Ray& r, Hits& xs, int depth = MAX_REFLECTION_ITERATIONS, Counters* k = nullptr) const {
        return internal_color_at(r, xs, depth, k);
    }
    // world.rs:114-128
    Color reflected_color(const Comps& c, Hits& xs, int remaining, Counters* k = nullptr) const {
        if (remaining == 0 || c.shape->material.reflectiveness == 0.0) return BLACK;
        if (k) k->reflect++;
        Ray rr{c.over_point, c.reflectv};
        return cscale(internal_color_at(rr, xs, remaining - 1, k), c.shape->material.reflectiveness);
    }
    // world.rs:130-157
    Color refracted_color(const Comps& c, Hits& xs, int remaining, Counters* k = nullptr) const {
        if (remaining == 0 || c.shape->material.transparency == 0.0) return BLACK;
        if (k) k->refract_evals++;
        double n_ratio = c.n1 / c.n2;
        double cos_i = dot(c.eye, c.normal);
        double sin2_t = sq(n_ratio) * (1.0 - sq(cos_i));
        if (sin2_t > 1.0) return BLACK;
        if (k) k->refract++;
        double cos_t = std::sqrt(1.0 - sin2_t);
        Vector dir = sub(scale(c.normal, std::fma(n_ratio, cos_i, -cos_t)), scale(c.eye, n_ratio));
        Ray rr{c.under_point, dir};
        return cscale(internal_color_at(rr, xs, remaining - 1, k), c.shape->material.transparency);
    }
};

// utils.rs:59-71 + world.rs:160-169
inline World default_world() {
    World w;
    w.lights.push_back({{-10, 10, -10}, WHITE});
    Shape s1;
    s1.material.color = {0.8, 1.0, 0.6};
    s1.material.diffuse = 0.7;
    s1.material.specular = 0.2;
    Shape s2;
    s2.set_transformation(scaling(0.5, 0.5, 0.5));
    w.shapes.push_back(s1);
    w.shapes.push_back(s2);
    return w;
}

// ------------------------------------------------------------------- camera
// camera.rs:9-19, 25-68, 114-127
struct Camera {
    uint32_t hsize = 0, vsize = 0;
    double fov = 0, half_width = 0, half_height = 0, pixel_size = 0;
    M4 inv = M4::identity();
    Point origin{0, 0, 0};

    Camera() = default;
    Camera(uint32_t h, uint32_t v, double field_of_view) : hsize(h), vsize(v), fov(field_of_view) {
        double half_view = std::tan(fov / 2.0);
        double aspect = (double)h / (double)v;
        if (aspect >= 1.0) {
            half_width = half_view;
            half_height = half_view / aspect;
        } else {
            half_width = half_view * aspect;
            half_height = half_view;
        }
        pixel_size = (half_width * 2.0) / (double)h;
    }
    void set_transformation(const M4& t) {
        inv = inverse(t);
        origin = mul_point(inv, Point{0, 0, 0});
    }
    Ray ray_for_pixel(uint32_t px, uint32_t py) const {
        double ox = ((double)px + 0.5) * pixel_size;
        double oy = ((double)py + 0.5) * pixel_size;
        double wx = half_width - ox;
        double wy = half_height - oy;
        Point pixel = mul_point(inv, Point{wx, wy, -1.0});
        Vector dir = normalized(sub(pixel, origin));
        return {origin, dir};
    }
};

// camera.rs:79-95 (serial) and 97-112 (rayon: per-pixel dynamic scheduling).
// Rows [row_begin, row_end) of the canvas, written row-major into out (3 f64).
inline void render_rows(const Camera& cam, const World& w, int depth, uint32_t row_begin, uint32_t row_end,
                        int threads, double* out, Counters* total) {
    const uint64_t W = cam.hsize;
    const uint64_t n = (uint64_t)(row_end - row_begin) * W;
    auto body = [&](uint64_t i, Hits& xs, Counters* k) {
        uint32_t x = (uint32_t)(i % W), y = row_begin + (uint32_t)(i / W);
        Ray r = cam.ray_for_pixel(x, y);
        if (k) k->primary++;
        Color c = w.color_at(r, xs, depth, k);
        out[3 * i + 0] = c.r;
        out[3 * i + 1] = c.g;
        out[3 * i + 2] = c.b;
    };
    if (threads <= 1) {
        Hits xs;
        Counters k;
        for (uint64_t i = 0; i < n; ++i) body(i, xs, &k);
        if (total) total->merge(k);
        return;
    }
    std::atomic<uint64_t> next{0};
    std::vector<Counters> ks(threads);
    std::vector<std::thread> pool;
    const uint64_t chunk = 64;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t]() {
            Hits xs;
            for (;;) {
                uint64_t b = next.fetch_add(chunk);
                if (b >= n) break;
                uint64_t e = std::min(n, b + chunk);
                for (uint64_t i = b; i < e; ++i) body(i, xs, &ks[t]);
            }
        });
    for (auto& th : pool) th.join();
    if (total)
        for (auto& k : ks) total->merge(k);
}

}  // namespace orc
