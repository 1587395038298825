"""Value identity of shapes, host side.

Value-equal shapes (shape.rs:34-38: same kind, derived field equality of
material, inverse transform and the kind's own fields) form one identity
class: the reference's containers walk toggles ONE list entry between them
(intersection.rs:47).  These CPU tests pin the host's class computation
through the YAML loader's count and show, on the oracle, that the rule
changes pixels (so the GPU test in test_gpu_identity.py is sensitive).
"""
import numpy as np


def dup_world(perturb=0.0):
    """World::default plus two value-equal glass spheres and two value-equal
    reflective planes (a duplicated floor).  `perturb` != 0 makes the second
    sphere's material differ in its last bits, so the pair is no longer equal."""
    from rtc_amd import world as W
    w = W.World.default()
    glass = dict(transparency=0.9, reflectiveness=0.9, refractive_index=1.5, ambient=0.05, diffuse=0.1,
                 color=(0.1, 0.1, 0.15))
    t = W.mat_mul(W.translation(0.4, 0.2, -1.6), W.scaling(0.6, 0.6, 0.6))
    w.shapes.append(W.sphere(W.Material(**glass), t))
    glass2 = dict(glass)
    glass2["ambient"] = glass["ambient"] + perturb
    w.shapes.append(W.sphere(W.Material(**glass2), [row[:] for row in t]))
    w.shapes.append(W.plane(W.Material(reflectiveness=0.3, color=(0.6, 0.7, 0.6)), W.translation(0, -1, 0)))
    w.shapes.append(W.plane(W.Material(reflectiveness=0.3, color=(0.6, 0.7, 0.6)), W.translation(0, -1, 0)))
    return w.tables()


DUP_YAML = """
- add: camera
  width: 8
  height: 6
  field-of-view: 1
  from: [0, 1, -5]
  to: [0, 0, 0]
  up: [0, 1, 0]
- add: light
  at: [-5, 5, -5]
  intensity: [1, 1, 1]
- define: glass-material
  value:
    transparency: 0.9
    refractive-index: 1.5
- add: sphere
  material: glass-material
  transform:
    - [translate, 0, 1, 0]
- add: sphere
  material: glass-material
  transform:
    - [translate, 0, 1, 0]
- add: sphere
  material: glass-material
  transform:
    - [translate, 0, 1.5, 0]
- add: plane
- add: plane
- add: cube
  material:
    color: [1, 0, 0]
- add: cube
  material:
    color: [1, 0, 0.0000001]
"""


def test_loader_counts_value_equal_shapes(rtc):
    t = rtc.load_scene_text(DUP_YAML)
    # sphere 2 equals sphere 1; plane 2 equals plane 1; the third sphere and
    # the second cube differ (transform / colour)
    assert t.duplicate_shapes == 2


def test_reference_scenes_have_no_value_equal_shapes(rtc):
    from conftest import scene_fixture
    for name in ("three_sphere_scene", "reflect_refract", "cover", "table", "cylinders", "metal", "refraction",
                 "shadow_puppets"):
        assert scene_fixture(name).duplicate_shapes == 0, name


def test_identity_rule_changes_the_image(oracle):
    """Equal pair vs a pair unequal in one material bit (invisible in the
    shading): the oracle's containers walk gives different refraction."""
    from rtc_amd import world as W
    cam = W.camera(48, 36, 0.9, (0, 0.6, -5), (0.2, 0, 0), (0, 1, 0))
    eq, _ = oracle.render(dup_world(), cam, 6, threads=8)
    ne, _ = oracle.render(dup_world(perturb=1e-15), cam, 6, threads=8)
    assert np.abs(eq - ne).max() > 1e-3
