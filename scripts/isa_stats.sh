#!/bin/bash
# Device ISA of the tracer kernels: register/LDS/spill metadata and
# instruction-class counts per kernel (CPU-side; no GPU needed).
set -e
OUT=${1:-/tmp/rtc_isa.s}
shift || true
cd "$(dirname "$0")/../ray-tracer-challenge-rs_amd"
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize --cuda-device-only -S "$@" \
    -o "$OUT" csrc/rtc_kernels.hip
python3 - "$OUT" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
for m in re.finditer(r"^(_ZN3rtc\w*trace_\w+):[^\n]*\n(.*?)^\s*s_endpgm", txt, re.S | re.M):
    name, body = m.group(1), m.group(2)
    ins = [l.strip().split()[0] for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    cnt = lambda p: sum(1 for i in ins if i.startswith(p))
    k = re.sub(r"EEEvNS_12Launch.*", "", name.replace("_ZN3rtc", ""))
    g = lambda f: (re.search(r"\.set " + re.escape(name) + r"\." + f + r", (\d+)", txt) or [None, "?"])[1]
    sec = (g("num_vgpr"), g("num_agpr"), g("numbered_sgpr"), g("private_seg_size"))
    print(f"{k:42s} ins={len(ins):5d} v_={cnt('v_'):5d} s_={cnt('s_'):5d} s_load={cnt('s_load'):4d} global_load={cnt('global_load'):4d} "
          f"ds_={cnt('ds_'):4d} cbranch={cnt('s_cbranch'):4d} scratch={cnt('scratch_'):3d} "
          f"vgpr/agpr/sgpr/priv={sec}")
PY
