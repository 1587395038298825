"""Host-side world construction mirroring the reference's public Rust API.

    primitives/transformations.rs  translation, scaling, rotation_{x,y,z}, shearing, view_transform
    composites/material.rs         Material (Default, glass)
    shapes/*.rs                    Sphere, Plane, Cube, Cylinder, Cone, Triangle
    patterns/*.rs                  Stripe/Gradient/Ring/Checker/Complex/Test patterns
    primitives/light.rs            Light
    composites/world.rs            World (+ World.default(), world.rs:160-169)
    composites/camera.rs           Camera(h, v, fov).set_transformation(...)

Matrices are 4x4 f64 nested lists combined with the reference's left-fold
product (matrix.rs:317-330) and inverted by the C++ host (rt_matrix_inverse,
the cofactor inverse of matrix.rs:247-258), so the tables handed to the GPU
carry exactly the reference's f64 values.  `World.tables(camera)` flattens
the trait-object world into the rt_* descriptor arrays.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

from . import (CameraDesc, LightDesc, MaterialDesc, PatternDesc, PATTERN_KINDS, SceneTables, ShapeDesc,
               SHAPE_KINDS, camera_make, matrix_inverse)

F64_MAX = 1.7976931348623157e308
IDENTITY = [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)]


def mat_mul(a, b):
    """Matrix<4> * Matrix<4>: left fold from 0.0, no FMA (matrix.rs:317-330)."""
    r = [[0.0] * 4 for _ in range(4)]
    for i in range(4):
        for j in range(4):
            acc = 0.0
            for k in range(4):
                acc = acc + a[i][k] * b[k][j]
            r[i][j] = acc
    return r


def translation(x, y, z):
    m = [row[:] for row in IDENTITY]
    m[0][3], m[1][3], m[2][3] = float(x), float(y), float(z)
    return m


def scaling(x, y, z):
    m = [row[:] for row in IDENTITY]
    m[0][0], m[1][1], m[2][2] = float(x), float(y), float(z)
    return m


def _rot(axis, theta):
    m = [row[:] for row in IDENTITY]
    c, s = math.cos(theta), math.sin(theta)
    if axis == 0:
        m[1][1], m[1][2], m[2][1], m[2][2] = c, -s, s, c
    elif axis == 1:
        m[0][0], m[0][2], m[2][0], m[2][2] = c, s, -s, c
    else:
        m[0][0], m[0][1], m[1][0], m[1][1] = c, -s, s, c
    return m


def rotation_x(t):
    return _rot(0, float(t))


def rotation_y(t):
    return _rot(1, float(t))


def rotation_z(t):
    return _rot(2, float(t))


def shearing(xy, xz, yx, yz, zx, zy):
    m = [row[:] for row in IDENTITY]
    m[0][1], m[0][2], m[1][0], m[1][2], m[2][0], m[2][1] = map(float, (xy, xz, yx, yz, zx, zy))
    return m


def inverse(m):
    return matrix_inverse([v for row in m for v in row]).tolist()


@dataclass
class Pattern:
    kind: str
    color_a: tuple = (1.0, 1.0, 1.0)
    color_b: tuple = (0.0, 0.0, 0.0)
    transformation_inverse: list = field(default_factory=lambda: [row[:] for row in IDENTITY])
    sub_a: "Pattern | None" = None
    sub_b: "Pattern | None" = None

    def set_transformation(self, m):
        self.transformation_inverse = inverse(m)
        return self


def stripe_pattern(a, b):
    return Pattern("stripe", tuple(a), tuple(b))


def gradient_pattern(a, b):
    return Pattern("gradient", tuple(a), tuple(b))


def ring_pattern(a, b):
    return Pattern("ring", tuple(a), tuple(b))


def checker_pattern(a, b):
    return Pattern("checker", tuple(a), tuple(b))


def complex_pattern(a: Pattern, b: Pattern):
    return Pattern("complex", sub_a=a, sub_b=b)


def test_pattern():
    return Pattern("test")


@dataclass
class Material:
    """material.rs:8-20; defaults material.rs:157-161."""
    color: tuple = (1.0, 1.0, 1.0)
    pattern: Pattern | None = None
    ambient: float = 0.1
    diffuse: float = 0.9
    specular: float = 0.9
    shininess: float = 200.0
    reflectiveness: float = 0.0
    refractive_index: float = 1.0
    transparency: float = 0.0
    casts_shadow: bool = True

    @staticmethod
    def glass() -> "Material":  # material.rs:148-154
        return Material(transparency=1.0, refractive_index=1.5)


@dataclass
class Shape:
    kind: str
    material: Material = field(default_factory=Material)
    transformation_inverse: list = field(default_factory=lambda: [row[:] for row in IDENTITY])
    minimum: float = -F64_MAX
    maximum: float = F64_MAX
    closed: bool = False
    triangle: tuple | None = None  # (v1, e1, e2, normal)

    def set_transformation(self, m):
        self.transformation_inverse = inverse(m)
        return self


def sphere(material=None, transform=None):
    s = Shape("sphere", material or Material())
    return s.set_transformation(transform) if transform is not None else s


def plane(material=None, transform=None):
    s = Shape("plane", material or Material())
    return s.set_transformation(transform) if transform is not None else s


def cube(material=None, transform=None):
    s = Shape("cube", material or Material())
    return s.set_transformation(transform) if transform is not None else s


def cylinder(minimum=-F64_MAX, maximum=F64_MAX, closed=False, material=None, transform=None):
    s = Shape("cylinder", material or Material(), minimum=float(minimum), maximum=float(maximum), closed=closed)
    return s.set_transformation(transform) if transform is not None else s


def cone(minimum=-F64_MAX, maximum=F64_MAX, closed=False, material=None, transform=None):
    s = Shape("cone", material or Material(), minimum=float(minimum), maximum=float(maximum), closed=closed)
    return s.set_transformation(transform) if transform is not None else s


def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def _cross(a, b):  # vector.rs:97-103 (mul_add: exact via math.fma when available)
    fma = getattr(math, "fma", None)
    if fma is None:  # Python < 3.13: emulate a correctly rounded fma through fractions
        from fractions import Fraction

        def fma(x, y, z):
            return float(Fraction(x) * Fraction(y) + Fraction(z))
    return (fma(a[1], b[2], -a[2] * b[1]), fma(a[2], b[0], -a[0] * b[2]), fma(a[0], b[1], -a[1] * b[0]))


def triangle(p1, p2, p3, material=None):
    """triangle.rs:21-35: edges and normal = normalize(e2 x e1)."""
    e1, e2 = _sub(p2, p1), _sub(p3, p1)
    n = _cross(e2, e1)
    mag = math.sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2])
    n = (n[0] / mag, n[1] / mag, n[2] / mag)
    return Shape("triangle", material or Material(), triangle=(tuple(map(float, p1)), e1, e2, n))


@dataclass
class Light:
    position: tuple
    intensity: tuple = (1.0, 1.0, 1.0)


@dataclass
class World:
    lights: list = field(default_factory=list)
    shapes: list = field(default_factory=list)

    @staticmethod
    def default() -> "World":
        """world.rs:160-169 with utils.rs:59-71."""
        s1 = sphere(Material(color=(0.8, 1.0, 0.6), diffuse=0.7, specular=0.2))
        s2 = sphere(transform=scaling(0.5, 0.5, 0.5))
        return World([Light((-10.0, 10.0, -10.0), (1.0, 1.0, 1.0))], [s1, s2])

    def tables(self, camera: CameraDesc | None = None) -> SceneTables:
        """Flatten into rt_* descriptor tables (one material entry per shape)."""
        pats: list[Pattern] = []

        def pat_index(p: Pattern | None) -> int:
            if p is None:
                return -1
            for i, q in enumerate(pats):
                if q is p:
                    return i
            pats.append(p)
            idx = len(pats) - 1
            if p.kind == "complex":
                pat_index(p.sub_a)
                pat_index(p.sub_b)
            return idx

        shapes = (ShapeDesc * len(self.shapes))()
        mats = (MaterialDesc * len(self.shapes))()
        for i, s in enumerate(self.shapes):
            d = shapes[i]
            d.kind = SHAPE_KINDS[s.kind]
            d.material = i
            d.inverse[:] = [float(v) for row in s.transformation_inverse for v in row]
            d.minimum, d.maximum, d.closed = s.minimum, s.maximum, int(s.closed)
            if s.triangle:
                d.vertex_1[:], d.edge_1[:], d.edge_2[:], d.normal[:] = [list(map(float, v)) for v in s.triangle]
            m, md = s.material, mats[i]
            md.color[:] = list(map(float, m.color))
            md.ambient, md.diffuse, md.specular, md.shininess = m.ambient, m.diffuse, m.specular, m.shininess
            md.reflectiveness, md.transparency, md.refractive_index = (m.reflectiveness, m.transparency,
                                                                       m.refractive_index)
            md.casts_shadow = int(m.casts_shadow)
            md.pattern = pat_index(m.pattern)
        ptab = (PatternDesc * len(pats))()
        for i, p in enumerate(pats):
            d = ptab[i]
            d.kind = PATTERN_KINDS[p.kind]
            d.color_a[:] = list(map(float, p.color_a))
            d.color_b[:] = list(map(float, p.color_b))
            d.inverse[:] = [float(v) for row in p.transformation_inverse for v in row]
            d.sub_a = pats.index(p.sub_a) if p.sub_a is not None else -1
            d.sub_b = pats.index(p.sub_b) if p.sub_b is not None else -1
        lts = (LightDesc * len(self.lights))()
        for i, lt in enumerate(self.lights):
            lts[i].position[:] = list(map(float, lt.position))
            lts[i].intensity[:] = list(map(float, lt.intensity))
        return SceneTables(shapes, mats, ptab, lts, camera if camera is not None else CameraDesc())


def camera(width, height, fov, frm=(0, 0, 0), to=(0, 0, -1), up=(0, 1, 0)) -> CameraDesc:
    """Camera::new(width, height, fov).set_transformation(view_transform(from, to, up))."""
    return camera_make(width, height, fov, frm, to, up)
