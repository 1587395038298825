"""Add the tables a newer kernel source expects (kMaterials; the shape clusters,
computed as rtc_jit.cpp make_clusters does) to a per-scene header dumped by an
older build (RTC_DEBUG=jit_dump=<dir>), from the scene's fixture, so scripts/jit_isa.sh can
compile it.  ISA inspection only.
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
if "kNumClusters" not in text:
    import math
    import re
    body = text[text.index("kShapes["):text.index("    {}};")]
    bounds = []
    for line in body.splitlines()[1:]:
        hx = re.findall(r"0x([0-9a-f]{8})u", line)
        if len(hx) >= 16:
            bounds.append([struct.unpack("<f", struct.pack("<I", int(h, 16)))[0] for h in hx[12:16]])
    bounded = [i for i, b in enumerate(bounds) if math.isfinite(b[3]) and b[3] >= 0]
    unclustered = [i for i in range(len(bounds)) if i not in bounded]
    balls, begin, members = [], [0], []
    if len(bounded) >= 6:
        k = min(6, max(2, round(math.sqrt(len(bounded)))))
        ctr = lambda i: bounds[i][:3]  # noqa: E731
        d2 = lambda a, b: sum((x - y) ** 2 for x, y in zip(a, b))  # noqa: E731
        cent = [ctr(bounded[0])]
        while len(cent) < k:
            cent.append(ctr(max(bounded, key=lambda i: min(d2(ctr(i), q) for q in cent))))
        lab = [0] * len(bounded)
        for _ in range(32):
            lab = [min(range(k), key=lambda q: d2(ctr(i), cent[q])) for i in bounded]
            for q in range(k):
                m = [ctr(bounded[j]) for j in range(len(bounded)) if lab[j] == q]
                if m:
                    cent[q] = [sum(c[t] for c in m) / len(m) for t in range(3)]
        for q in range(k):
            m = [bounded[j] for j in range(len(bounded)) if lab[j] == q]
            if not m:
                continue
            r = max(math.sqrt(d2(ctr(i), cent[q])) + math.sqrt(bounds[i][3]) for i in m)
            pad = 1e-4 * (r + sum(abs(c) for c in cent[q])) + 1e-4
            balls.append(cent[q] + [(r + pad) ** 2])
            members += m
            begin.append(len(members))
    else:
        unclustered = list(range(len(bounds)))

    def f(v):
        return "__builtin_bit_cast(float, 0x%08xu)" % struct.unpack("<I", struct.pack("<f", v))[0]
    ints = lambda v: "{" + ", ".join(map(str, v or [0])) + "}"  # noqa: E731
    add = "constexpr int kNumClusters = %d;\n" % len(balls)
    add += "constexpr float kClusterBall[%d][4] = {\n%s    {}};\n" % (
        len(balls) + 1, "".join("    {%s},\n" % ", ".join(f(x) for x in b) for b in balls))
    add += "constexpr int kClusterBegin[%d] = %s;\n" % (len(begin), ints(begin))
    add += "constexpr int kClusterMembers[%d] = %s;\n" % (max(1, len(members)), ints(members))
    add += "constexpr int kNumUnclustered = %d;\n" % len(unclustered)
    add += "constexpr int kUnclustered[%d] = %s;\n" % (max(1, len(unclustered)), ints(unclustered))
    text = text.replace("constexpr int kNumLights", add + "constexpr int kNumLights", 1)
sys.stdout.write(text)
