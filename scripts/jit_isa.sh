#!/bin/bash
# Device ISA of a per-scene (hipRTC) build, made here with hipcc from a scene
# header dumped on the GPU box (RTC_DEBUG=jit_dump=<dir>: <key>_direct.hpp /
# <key>_pool.hpp).  Same source, defines and flags as rtc_jit.cpp
# make_request; prints the instruction-class counts of scripts/isa_stats.sh.
#   scripts/jit_isa.sh <scene.hpp> [out.s] [extra hipcc flags...]
set -e
HPP=$(realpath "$1")
OUT=$(realpath -m "${2:-/tmp/rtc_jit_isa.s}")
shift; [ $# -gt 0 ] && shift
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
mkdir -p "$T/a/b" "$T/include"
cp "$HPP" "$T/a/b/rtc_jit_scene.hpp"
cp "$ROOT/ray-tracer-challenge-rs_amd/csrc/rtc_internal.hpp" "$T/a/b/"
cp "$ROOT/include/rtc.h" "$T/include/"
EXTRA_DEF=
KERNEL=${JIT_KERNEL:-"trace_pool<float, true, false>"}
case "$HPP" in *_direct.hpp) EXTRA_DEF=-DRTC_JIT_FENCE_EVERY=3; KERNEL=${JIT_KERNEL:-"trace_direct<float, false>"} ;; esac
# hipRTC instantiates the kernel from its name expression; here explicitly
{ printf '#define RTC_JIT 1\n#include "rtc_jit_scene.hpp"\n'; cat "$ROOT/ray-tracer-challenge-rs_amd/csrc/rtc_kernels.hip"
  printf '\nnamespace rtc {\ntemplate __global__ void %s(LaunchParams<float>, RTC_WORLD_PARAMS(float));\n}\n' "$KERNEL"; } > "$T/a/b/k.hip"
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
    -mllvm -disable-machine-licm $EXTRA_DEF "$@" --cuda-device-only -S -o "$OUT" "$T/a/b/k.hip"
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
    print(f"{k:42s} ins={len(ins):5d} v_={cnt('v_'):5d} s_={cnt('s_'):5d} s_load={cnt('s_load'):4d} "
          f"ds_={cnt('ds_'):4d} cbranch={cnt('s_cbranch'):4d} scratch={cnt('scratch_'):3d} "
          f"vgpr/agpr/sgpr/priv={sec}")
PY
