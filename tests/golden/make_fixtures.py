"""Generate the committed fixtures under tests/golden/ from the reference
checkout (/root/reference, build container only).

  scenes/<name>.json   the reference's scenes/<name>.yaml flattened by OUR
                       loader (rt_scene_load_yaml, scene_loader.rs semantics)
                       into the rt_* descriptor tables + camera.  The loader
                       itself is checked against an independent PyYAML
                       restatement in tests/test_loader.py.
  png_bands.npz        two 8-row bands of each reference render
                       (rendered_images/<name>.png, 8-bit, native size): the
                       expected outputs the oracle must reproduce
                       (tests/test_oracle_images.py).

Usage: python tests/golden/make_fixtures.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "ray-tracer-challenge-rs_amd"))

import rtc_amd  # noqa: E402
from rtc_amd import scene_io  # noqa: E402

SCENES = ["three_sphere_scene", "reflect_refract", "cover", "table", "cylinders", "metal", "refraction",
          "shadow_puppets"]
BAND_ROWS = 8


def band_starts(height: int):
    return [height // 3 // BAND_ROWS * BAND_ROWS, (2 * height) // 3 // BAND_ROWS * BAND_ROWS]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    from PIL import Image

    os.makedirs(os.path.join(HERE, "scenes"), exist_ok=True)
    bands = {}
    for name in SCENES:
        src = os.path.join(args.reference, "scenes", f"{name}.yaml")
        scene = rtc_amd.load_scene(src)
        scene_io.save(scene, os.path.join(HERE, "scenes", f"{name}.json"), source=f"scenes/{name}.yaml")
        png = np.asarray(Image.open(os.path.join(args.reference, "rendered_images", f"{name}.png")).convert("RGB"))
        assert png.shape[:2] == (scene.camera.height, scene.camera.width), (name, png.shape)
        for r0 in band_starts(scene.camera.height):
            bands[f"{name}@{r0}"] = png[r0:r0 + BAND_ROWS].copy()
        print(name, scene.counts, png.shape)
    np.savez_compressed(os.path.join(HERE, "png_bands.npz"), **bands)


if __name__ == "__main__":
    main()
