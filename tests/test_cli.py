"""The `rtc` CLI (csrc/rtc_cli.cpp): the reference CLI's flow (main.rs:11-31,
cli_arguments.rs:4-13) over the C-ABI — YAML in, 8-bit image out."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG

CLI = os.path.join(PKG, "rtc_amd", "_lib", "rtc")

SCENE = """
- add: camera
  width: 64
  height: 48
  field-of-view: 0.9
  from: [0, 1.5, -5]
  to: [0, 1, 0]
  up: [0, 1, 0]
- add: light
  at: [-10, 10, -10]
  intensity: [1, 1, 1]
- add: plane
  material:
    pattern:
      type: checkers
      colors:
        - [1, 1, 1]
        - [0.1, 0.1, 0.1]
    reflective: 0.3
- add: sphere
  transform:
    - [translate, -0.5, 1, 0.5]
  material:
    color: [0.1, 0.2, 0.3]
    transparency: 0.9
    reflective: 0.9
    refractive-index: 1.5
- add: cube
  transform:
    - [scale, 0.4, 0.4, 0.4]
    - [translate, 1.5, 0.4, -0.5]
  material:
    color: [1, 0.3, 0.2]
"""


def read_ppm(path, magic=b"P3"):
    """The CLI saves .ppm as the reference's P3 text (canvas.rs:75-97); P6 with --ppm-binary."""
    data = open(path, "rb").read()
    parts = data.split(b"\n", 3)
    assert parts[0] == magic and parts[2] == b"255"
    w, h = map(int, parts[1].split())
    if magic == b"P6":
        return np.frombuffer(parts[3], dtype=np.uint8).reshape(h, w, 3)
    lines = parts[3].split(b"\n")
    assert not data.endswith(b"\n") and all(len(x) == 15 * 4 - 1 for x in lines[:-1])
    return np.array(parts[3].split(), dtype=np.int64).astype(np.uint8).reshape(h, w, 3)


def test_cli_usage_and_missing_scene_fail_loudly(tmp_path):
    r = subprocess.run([CLI], capture_output=True, text=True)
    # -r serial|parallel render on the GPU too, and the help says so (no CPU renderer ships)
    assert r.returncode != 0 and "no CPU renderer" in r.stderr
    assert subprocess.run([CLI, "a.yaml", "b.png", "-r", "bogus"], capture_output=True).returncode == 2
    r = subprocess.run([CLI, str(tmp_path / "missing.yaml"), str(tmp_path / "o.ppm")], capture_output=True, text=True)
    assert r.returncode != 0 and "error" in r.stderr


@pytest.mark.gpu
def test_cli_renders_the_scene_like_the_oracle(tmp_path, rtc, oracle):
    yaml = tmp_path / "scene.yaml"
    yaml.write_text(SCENE)
    out = tmp_path / "out.ppm"
    r = subprocess.run([CLI, str(yaml), str(out), "--precision", "f64", "--width", "80", "--height", "60"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Image rendered in" in r.stdout
    img = read_ppm(out)
    scene = rtc.load_scene(str(yaml))
    ref, _ = oracle.render(scene, rtc.camera_resize(scene.camera, 80, 60), 6)
    d = np.abs(img.astype(int) - oracle.quantize(ref).astype(int))
    assert d.max() <= 1 and (d == 0).mean() >= 0.999


@pytest.mark.gpu
def test_cli_png_equals_ppm(tmp_path):
    """`rtc scene.yaml out.png` saves the same pixels as PNG (main.rs:26,
    canvas.rs:114-137) that `out.ppm` saves as PPM."""
    PIL = pytest.importorskip("PIL.Image")
    yaml = tmp_path / "scene.yaml"
    yaml.write_text(SCENE)
    outs = {}
    for ext, mode in (("ppm", "parallel"), ("png", "serial")):  # the reference's -r modes: same GPU render
        out = tmp_path / f"out.{ext}"
        r = subprocess.run([CLI, str(yaml), str(out), "-r", mode, "--width", "64", "--height", "48"],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert f"Image saved at {out}" in r.stdout  # main.rs:27-29
        outs[ext] = out
    with PIL.open(outs["png"]) as im:
        assert np.array_equal(np.asarray(im.convert("RGB")), read_ppm(outs["ppm"]))
    out = tmp_path / "out_p6.ppm"
    r = subprocess.run([CLI, str(yaml), str(out), "--ppm-binary", "-q", "--width", "64", "--height", "48"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(read_ppm(out, b"P6"), read_ppm(outs["ppm"]))
