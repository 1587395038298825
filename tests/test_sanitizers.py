"""ASan + UBSan runs of the host-only C++ ("Host: ASan/UBSan
builds of the C++ oracle and host").  The reference gets this from Rust
("No `unsafe` code", README.md:14); here the hand-written YAML tokenizer
(csrc/scene_loader.cpp), the PNG/PPM writers (csrc/image_io.cpp), the
per-scene build cache files (csrc/rtc_jit_cache.hpp) and the f64 oracle
(oracle/) run under g++ -fsanitize=address,undefined with
-fno-sanitize-recover, so any report fails the test (tests/sanitize/).

* the oracle's KAT runner: its output equals the optimised build's, byte for byte;
* scenes: a feature-complete YAML scene plus the loader tests' documents (and
  the reference's own scenes/*.yaml where /root/reference is mounted) are
  loaded, rendered by the oracle, quantized and written as PNG, P3 and P6;
* fuzzing: seeded byte mutations of those documents (deletions, insertions,
  bit flips, duplicated spans, truncations) through the loader and the oracle;
* the code-object and request files: every truncation and random bit flips;
* canvas quantization of NaN / inf / edge values and image writes of
  degenerate sizes and unwritable paths.
"""
import glob
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = os.path.join(HERE, "sanitize")
BUILD = os.path.join(SAN, "_build")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")

# every loader feature the reference scenes use (scene_loader.rs:46-335)
KITCHEN_SINK = """
- add: camera
  width: 24
  height: 16
  field-of-view: 1.0472
  from: [0, 1.5, -5]
  to: [0, 1, 0]
  up: [0, 1, 0]
- add: light
  at: [-10, 10, -10]
  intensity: [1, 1, 1]
- add: light
  at: [5, 8, -6]
  intensity: [0.3, 0.3, 0.4]
- define: white-material
  value:
    color: [1, 1, 1]
    diffuse: 0.7
    ambient: 0.1
    specular: 0.0
    reflective: 0.1
- define: blue-material
  extend: white-material
  value:
    color: [0.537, 0.831, 0.914]
- define: glass-material
  value:
    color: [0.1, 0.1, 0.1]
    transparency: 0.9
    reflective: 0.9
    refractive-index: 1.5
    casts-shadow: false
- define: standard-transform
  value:
    - [translate, 1, -1, 1]
    - [scale, 0.5, 0.5, 0.5]
- define: large-object
  value:
    - standard-transform
    - [scale, 3.5, 3.5, 3.5]
- add: plane
  material:
    pattern:
      type: checkers
      colors:
        - [0.35, 0.35, 0.35]
        - [0.65, 0.65, 0.65]
    reflective: 0.4
- add: plane
  transform:
    - [rotate-x, 1.5708]
    - [translate, 0, 0, 10]
  material:
    pattern:
      type: stripes
      colors:
        - [1, 0, 0]
        - [0, 0, 1]
      transform:
        - [rotate-y, 0.3]
        - [scale, 0.25, 0.25, 0.25]
- add: sphere
  transform:
    - [scale, 0.7, 0.7, 0.7]
    - [translate, 0.6, 0.7, -0.6]
  material: glass-material
- add: sphere
  transform:
    - [translate, -1.5, 0.5, 1]
  material:
    pattern:
      type: rings
      colors:
        - [1, 1, 0]
        - [0, 1, 0]
- add: sphere
  transform:
    - [translate, 2, 0.5, 2]
  material:
    pattern:
      type: gradient
      colors:
        - [1, 0, 0]
        - [0, 0, 1]
- add: cube
  transform:
    - large-object
    - [rotate-y, 0.4]
    - [shear, 0.1, 0, 0, 0, 0, 0]
  material: blue-material
- add: cylinder
  min: 0
  max: 1.5
  closed: true
  transform:
    - [translate, -3, 0, 3]
  material: white-material
- add: cone
  min: -1
  max: 0
  closed: true
  transform:
    - [translate, 3, 1, 4]
- add: cylinder
  transform:
    - [scale, 0.2, 1, 0.2]
    - [translate, 4, 0, 6]
"""

LOADER_DOCS = [
    "- add: camera\n  width: 8\n  height: 6\n  field-of-view: 1.0\n  from: [0, 0, -5]\n  to: [0, 0, 0]\n"
    "  up: [0, 1, 0]\n- add: light\n  at: [.0, 1.0, 1]\n  intensity: [1, 1, 1]\n- add: triangle\n- add: group\n"
    "- add: sphere\n  transform:\n    - [translate, 1, 0, 0]\n",
]


def _build():
    subprocess.run(["make", "-s", "-C", SAN, "-j4"], check=True)


@pytest.fixture(scope="module")
def san():
    _build()
    return os.path.join(BUILD, "san_driver")


def _run(cmd, tmp_path):
    env = dict(ENV, SAN_TMP=str(tmp_path))
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, \
        (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def _scene_files(tmp_path):
    paths = []
    for i, text in enumerate([KITCHEN_SINK] + LOADER_DOCS):
        p = tmp_path / f"doc{i}.yaml"
        p.write_text(text)
        paths.append(str(p))
    paths += sorted(glob.glob("/root/reference/scenes/*.yaml"))  # input data, where mounted
    return paths


def test_oracle_kats_under_sanitizers(san, tmp_path):
    kat = os.path.join(ROOT, "oracle", "_build", "kat_runner")
    if not os.path.exists(kat):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    want = subprocess.run([kat], capture_output=True, text=True, check=True).stdout
    got = _run([os.path.join(BUILD, "kat_runner_san")], tmp_path)
    assert got == want


def test_scenes_load_render_write_under_sanitizers(san, tmp_path):
    out = _run([san, "scene"] + _scene_files(tmp_path), tmp_path)
    assert "loaded and rendered" in out
    assert (tmp_path / "san_scene.png").stat().st_size > 0


def test_fuzzed_scenes_under_sanitizers(san, tmp_path):
    files = _scene_files(tmp_path)[:2]
    out = _run([san, "fuzz", "400", "20261017"] + files, tmp_path)
    assert "mutated scenes loaded" in out


def test_jit_cache_files_under_sanitizers(san, tmp_path):
    out = _run([san, "jitcache", "400", "7"], tmp_path)
    assert "flipped files still parsed" in out


def test_images_under_sanitizers(san, tmp_path):
    assert "images: ok" in _run([san, "images"], tmp_path)
