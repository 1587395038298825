"""Flattened scene tables <-> JSON.

The reference's YAML scenes are only readable in the build container; the GPU
box gets them as the descriptor tables our loader produced (rt_scene_load_yaml,
scene_loader.rs semantics), written with exact float repr so every f64
round-trips bit-for-bit.  tests/golden/make_fixtures.py writes these files.
"""
from __future__ import annotations

import json

from . import CameraDesc, LightDesc, MaterialDesc, PatternDesc, SceneTables, ShapeDesc


def _struct_to_dict(s) -> dict:
    out = {}
    for name, typ in s._fields_:
        v = getattr(s, name)
        out[name] = list(v) if hasattr(v, "__len__") and not isinstance(v, (str, bytes)) else v
    return out


def _dict_to_struct(cls, d: dict):
    s = cls()
    for name, typ in cls._fields_:
        if name not in d:
            continue
        v = d[name]
        if isinstance(v, list):
            getattr(s, name)[:] = v
        else:
            setattr(s, name, v)
    return s


def tables_to_dict(scene: SceneTables) -> dict:
    return {
        "shapes": [_struct_to_dict(x) for x in scene.shapes],
        "materials": [_struct_to_dict(x) for x in scene.materials],
        "patterns": [_struct_to_dict(x) for x in scene.patterns],
        "lights": [_struct_to_dict(x) for x in scene.lights],
        "camera": _struct_to_dict(scene.camera),
        "duplicate_shapes": scene.duplicate_shapes,
    }


def tables_from_dict(d: dict) -> SceneTables:
    def arr(cls, items):
        a = (cls * len(items))()
        for i, it in enumerate(items):
            a[i] = _dict_to_struct(cls, it)
        return a
    return SceneTables(arr(ShapeDesc, d["shapes"]), arr(MaterialDesc, d["materials"]),
                       arr(PatternDesc, d["patterns"]), arr(LightDesc, d["lights"]),
                       _dict_to_struct(CameraDesc, d["camera"]), d.get("duplicate_shapes", 0))


def save(scene: SceneTables, path: str, source: str = "") -> None:
    d = tables_to_dict(scene)
    d["_source"] = source
    with open(path, "w") as f:
        json.dump(d, f, indent=1)


def load(path: str) -> SceneTables:
    with open(path) as f:
        return tables_from_dict(json.load(f))
