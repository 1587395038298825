// host_math.hpp — f64 host-side precompute of the render path: the parts of
// the reference that run once per scene/frame on the host and therefore stay
// f64 on the host here:
//   Matrix<4> product / cofactor inverse   primitives/matrix.rs:189-259, 317-346
//   transformation builders                primitives/transformations.rs:5-87
//   Camera::new / set_transformation       composites/camera.rs:25-49, 114-127
// Operation order matches the reference (left folds from 0.0, cofactor
// expansion along row 0, the is_identity shortcuts), so the matrices handed
// to the device are bit-identical to the reference's.  Compiled with
// -ffp-contract=off.
#pragma once

#include <cfloat>
#include <cmath>
#include <cstdint>

namespace rtc {
namespace hm {

constexpr double EPSILON = 0.00000008;  // consts.rs:2

struct M4 {
    double m[4][4];
};

inline M4 identity() {
    M4 r{};
    for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0;
    return r;
}

inline bool near(double a, double b) { return a == b || std::fabs(a - b) < EPSILON; }  // utils.rs:16-24

template <int N>
inline bool is_identity_n(const double (*a)[N]) {  // matrix.rs:45-51
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j)
            if (!near(a[i][j], i == j ? 1.0 : 0.0)) return false;
    return true;
}

inline M4 mul(const M4& a, const M4& b) {  // matrix.rs:317-330
    M4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 4; ++k) acc = acc + a.m[i][k] * b.m[k][j];
            r.m[i][j] = acc;
        }
    return r;
}

inline void mul_point(const M4& a, const double p[3], double out[3]) {  // matrix.rs:332-346
    const double v[4] = {p[0], p[1], p[2], 1.0};
    for (int r = 0; r < 3; ++r) {
        double acc = 0.0;
        for (int c = 0; c < 4; ++c) acc = acc + a.m[r][c] * v[c];
        out[r] = acc;
    }
}

// --- cofactor inverse, matrix.rs:65-259 -------------------------------------
inline double det2(double a, double b, double c, double d) { return (a * d) - (b * c); }

struct M3 {
    double m[3][3];
};

inline double cof3(const M3& a, int row, int col);
inline double det3(const M3& a) {
    double acc = 0.0;
    for (int i = 0; i < 3; ++i) acc = acc + a.m[0][i] * cof3(a, 0, i);
    return acc;
}
inline double cof3(const M3& a, int row, int col) {
    double s[2][2];
    for (int i = 0, ri = 0; i < 3; ++i) {
        if (i == row) continue;
        for (int j = 0, cj = 0; j < 3; ++j) {
            if (j == col) continue;
            s[ri][cj++] = a.m[i][j];
        }
        ++ri;
    }
    double minor = det2(s[0][0], s[0][1], s[1][0], s[1][1]);
    return ((row + col) % 2 == 0) ? minor : -minor;
}
inline double cof4(const M4& a, int row, int col) {
    M3 s{};
    if (is_identity_n<4>(a.m)) {  // Matrix<4>::submatrix shortcut, matrix.rs:192-194
        for (int i = 0; i < 3; ++i) s.m[i][i] = 1.0;
    } else {
        for (int i = 0, ri = 0; i < 4; ++i) {
            if (i == row) continue;
            for (int j = 0, cj = 0; j < 4; ++j) {
                if (j == col) continue;
                s.m[ri][cj++] = a.m[i][j];
            }
            ++ri;
        }
    }
    double minor = det3(s);
    return ((row + col) % 2 == 0) ? minor : -minor;
}
inline double det4(const M4& a) {
    double acc = 0.0;
    for (int i = 0; i < 4; ++i) acc = acc + a.m[0][i] * cof4(a, 0, i);
    return acc;
}
inline M4 inverse(const M4& a) {  // matrix.rs:247-258
    if (is_identity_n<4>(a.m)) return identity();
    M4 r{};
    const double det = det4(a);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.m[i][j] = cof4(a, j, i) / det;
    return r;
}

// --- builders, transformations.rs:5-87 ---------------------------------------
inline M4 translation(double x, double y, double z) {
    M4 r = identity();
    r.m[0][3] = x;
    r.m[1][3] = y;
    r.m[2][3] = z;
    return r;
}
inline M4 scaling(double x, double y, double z) {
    M4 r = identity();
    r.m[0][0] = x;
    r.m[1][1] = y;
    r.m[2][2] = z;
    return r;
}
inline M4 rotation(int axis, double theta) {
    M4 r = identity();
    const double c = std::cos(theta), s = std::sin(theta);
    if (axis == 0) {
        r.m[1][1] = c; r.m[1][2] = -s; r.m[2][1] = s; r.m[2][2] = c;
    } else if (axis == 1) {
        r.m[0][0] = c; r.m[0][2] = s; r.m[2][0] = -s; r.m[2][2] = c;
    } else {
        r.m[0][0] = c; r.m[0][1] = -s; r.m[1][0] = s; r.m[1][1] = c;
    }
    return r;
}

// vector.rs:84-103 (dot/cross fused exactly where the reference writes mul_add)
inline void normalize3(const double v[3], double out[3]) {
    const double mag = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    out[0] = v[0] / mag;
    out[1] = v[1] / mag;
    out[2] = v[2] / mag;
}
inline void cross3(const double a[3], const double b[3], double out[3]) {
    out[0] = std::fma(a[1], b[2], -a[2] * b[1]);
    out[1] = std::fma(a[2], b[0], -a[0] * b[2]);
    out[2] = std::fma(a[0], b[1], -a[1] * b[0]);
}

inline M4 view_transform(const double from[3], const double to[3], const double up[3]) {
    const double d[3] = {to[0] - from[0], to[1] - from[1], to[2] - from[2]};
    double fwd[3], upn[3], left[3], tup[3];
    normalize3(d, fwd);
    normalize3(up, upn);
    cross3(fwd, upn, left);
    cross3(left, fwd, tup);
    M4 o{};
    o.m[0][0] = left[0]; o.m[0][1] = left[1]; o.m[0][2] = left[2];
    o.m[1][0] = tup[0]; o.m[1][1] = tup[1]; o.m[1][2] = tup[2];
    o.m[2][0] = -fwd[0]; o.m[2][1] = -fwd[1]; o.m[2][2] = -fwd[2];
    o.m[3][3] = 1.0;
    return mul(o, translation(-from[0], -from[1], -from[2]));
}

// Camera::new, camera.rs:25-49
struct CameraSize {
    double half_width, half_height, pixel_size;
};
inline CameraSize camera_size(uint32_t w, uint32_t h, double fov) {
    const double half_view = std::tan(fov / 2.0);
    const double aspect = (double)w / (double)h;
    CameraSize s;
    if (aspect >= 1.0) {
        s.half_width = half_view;
        s.half_height = half_view / aspect;
    } else {
        s.half_width = half_view * aspect;
        s.half_height = half_view;
    }
    s.pixel_size = (s.half_width * 2.0) / (double)w;
    return s;
}

}  // namespace hm
}  // namespace rtc
