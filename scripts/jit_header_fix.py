"""Add the tables a newer kernel source expects (kMaterials) to a per-scene
header dumped by an older build (RTC_JIT_DUMP), from the scene's fixture, so
scripts/jit_isa.sh can compile it.  ISA inspection only.
Usage: python scripts/jit_header_fix.py <dumped.hpp> <scene name> > fixed.hpp"""
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hpp, name = sys.argv[1], sys.argv[2]
text = open(hpp).read()
if "kMaterials" not in text:
    mats = json.load(open(os.path.join(ROOT, "tests", "golden", "scenes", f"{name}.json")))["materials"]

    def f(v):
        return "__builtin_bit_cast(float, 0x%08xu)" % struct.unpack("<I", struct.pack("<f", v))[0]
    rows = []
    for m in mats:
        vals = [f(c) for c in m["color"]] + [f(m[k]) for k in ("ambient", "diffuse", "specular", "shininess",
                                                                "reflectiveness", "transparency", "refractive_index")]
        rows.append("    {{%s, %s, %s}, %s, %d, %d}," % (vals[0], vals[1], vals[2], ", ".join(vals[3:]), m["pattern"],
                                                     m["casts_shadow"]))
    table = "constexpr MaterialRec<float> kMaterials[%d] = {\n%s\n    {}};\n" % (len(mats) + 1, "\n".join(rows))
    text = text.replace("constexpr bool kPatterns", table + "constexpr bool kPatterns", 1)
sys.stdout.write(text)
