"""The Rust shim's #[repr(C)] mirrors against include/rtc.h.

There is no Rust toolchain in this image, so the shim is source only.  This
test pins what a compiler would otherwise catch at the FFI seam: every
`#[repr(C)] pub struct Rt*` in INTEGRATION.md is parsed, laid out by the
repr(C) rules (fields in order, each at the next multiple of its alignment,
size rounded to the struct's alignment), and compared field by field —
name, offset and size — with the C header's own layout, which gcc reports
for a generated offsetof() program compiled against include/rtc.h.  The same
C layout is also compared with the ctypes mirror in rtc_amd.  The functions
the shim declares in `extern "C"` must be declared by the header.
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT

INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")
RUST_PRIM = {"i32": (4, 4), "u32": (4, 4), "u64": (8, 8), "i64": (8, 8), "f64": (8, 8), "f32": (4, 4),
             "u8": (1, 1)}


def _rust_source():
    text = open(INTEGRATION).read()
    blocks = re.findall(r"```rust\n(.*?)```", text, re.S)
    assert blocks, "INTEGRATION.md has no rust code block"
    return "\n".join(blocks)


def _rust_type(t):
    t = t.strip()
    m = re.fullmatch(r"\[(\w+);\s*(\d+)\]", t)
    if m:
        size, align = RUST_PRIM[m.group(1)]
        return size * int(m.group(2)), align
    return RUST_PRIM[t]


def _rust_structs():
    out = {}
    for name, body in re.findall(r"#\[repr\(C\)\][^\n]*\n?\s*pub struct (Rt\w+)\s*\{(.*?)\}", _rust_source(), re.S):
        fields, off, salign = [], 0, 1
        for decl in body.split(","):
            decl = decl.strip()
            if not decl:
                continue
            fname, ftype = decl.replace("pub ", "").split(":", 1)
            size, align = _rust_type(ftype)
            off = (off + align - 1) // align * align
            fields.append((fname.strip(), off, size))
            off += size
            salign = max(salign, align)
        out[name] = (fields, (off + salign - 1) // salign * salign)
    return out


def _c_name(rust_name):  # RtShapeDesc -> rt_shape_desc
    return re.sub(r"(?<!^)(?=[A-Z])", "_", rust_name).lower()


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    structs = {k: v for k, v in _rust_structs().items() if v[0] and not v[0][0][0].startswith("_")}
    lines = ["#include <stddef.h>", "#include <stdio.h>", '#include "rtc.h"', "int main(void) {"]
    for rname, (fields, _) in structs.items():
        c = _c_name(rname)
        lines.append(f'  printf("{rname} sizeof %zu\\n", sizeof({c}));')
        for f, _, _ in fields:
            lines.append(f'  printf("{rname} {f} %zu %zu\\n", offsetof({c}, {f}), sizeof((({c}*)0)->{f}));')
    lines.append("  return 0; }")
    d = tmp_path_factory.mktemp("layout")
    src, exe = d / "layout.c", d / "layout"
    src.write_text("\n".join(lines) + "\n")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)],
                   check=True)
    out = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        parts = line.split()
        if parts[1] == "sizeof":
            out[(parts[0], None)] = int(parts[2])
        else:
            out[(parts[0], parts[1])] = (int(parts[2]), int(parts[3]))
    return structs, out


def test_shim_declares_every_descriptor():
    names = set(_rust_structs())
    for n in ("RtShapeDesc", "RtMaterialDesc", "RtPatternDesc", "RtLightDesc", "RtCameraDesc", "RtRenderOptions",
              "RtStats"):
        assert n in names, n


def test_repr_c_layout_matches_the_header(c_layout):
    structs, c = c_layout
    for rname, (fields, size) in structs.items():
        assert c[(rname, None)] == size, f"{rname}: Rust size {size}, C size {c[(rname, None)]}"
        for f, off, fsize in fields:
            assert c[(rname, f)] == (off, fsize), f"{rname}.{f}: Rust ({off}, {fsize}) vs C {c[(rname, f)]}"


def test_ctypes_mirror_matches_the_header(c_layout, rtc):
    import ctypes as C
    structs, c = c_layout
    mirror = {"RtShapeDesc": rtc.ShapeDesc, "RtMaterialDesc": rtc.MaterialDesc, "RtPatternDesc": rtc.PatternDesc,
              "RtLightDesc": rtc.LightDesc, "RtCameraDesc": rtc.CameraDesc, "RtRenderOptions": rtc.RenderOptions,
              "RtStats": rtc.Stats}
    for rname, cls in mirror.items():
        assert C.sizeof(cls) == c[(rname, None)], rname
        for fname, _ in cls._fields_:
            assert getattr(cls, fname).offset == c[(rname, fname)][0], f"{rname}.{fname}"


def test_shim_functions_are_declared_by_the_header():
    src = _rust_source()
    ext = re.search(r'extern "C"\s*\{(.*?)\n\}', src, re.S).group(1)
    header = open(os.path.join(ROOT, "include", "rtc.h")).read() + open(os.path.join(ROOT, "include",
                                                                                         "rtc_scene.h")).read()
    fns = re.findall(r"fn (rt_\w+)\(", ext)
    assert fns
    for f in fns:
        assert re.search(r"\b" + f + r"\(", header), f
