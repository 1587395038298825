"""Secondary whole-image pin of the oracle: the reference's own committed
renders (rendered_images/*.png, native resolution, 8-bit via canvas.rs:117-123)
against the oracle rendering the same rows of the same YAML scene.

The fixture (tests/golden/png_bands.npz, made by tests/golden/make_fixtures.py)
holds two 8-row bands per image (16 bands, 8 scenes, 491 520 pixels).  The
provenance of those PNGs relative to the reference's current code is
unverified, yet the oracle reproduces every band bit-exactly,
so the test demands exactly that: it pins the whole render path (loader,
camera, every shape and pattern the scenes use, shading, recursion, Schlick,
quantization) at the reference's native resolutions.
"""
import numpy as np
import pytest

from conftest import GOLDEN, scene_fixture

BANDS = np.load(f"{GOLDEN}/png_bands.npz")
KEYS = sorted(BANDS.files)
BAND_ROWS = 8


@pytest.mark.parametrize("key", KEYS)
def test_oracle_matches_reference_png_band(oracle, key):
    name, r0 = key.split("@")
    r0 = int(r0)
    png = BANDS[key]
    scene = scene_fixture(name)
    cam = scene.camera
    assert png.shape == (BAND_ROWS, cam.width, 3), "fixture and scene camera disagree on the image width"
    img, _ = oracle.render(scene, cam, 6, rows=(r0, r0 + BAND_ROWS), threads=8)
    q = oracle.quantize(img).astype(int)
    diff = np.abs(q - png.astype(int)).max(axis=2)
    assert diff.max() == 0, f"{key}: {int((diff > 0).sum())} pixels differ from the reference PNG, max {diff.max()}/255"
