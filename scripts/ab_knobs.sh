#!/bin/bash
# Same-box A/B of RTC_DEBUG settings (csrc/debug_knobs.hpp), alternating
# ROUNDS times over the listed workloads:
#   scripts/ab_knobs.sh "name=RTC_DEBUG value" ...   ("base=" = none)
# WORKLOADS: ';'-separated bench.py argument sets.  One JSON line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
IFS=';' read -ra WL <<< "${WORKLOADS:---scene reflect_refract --steps 300;--scene cover --width 3840 --height 2160 --steps 100;--scene table --width 3840 --height 2160 --steps 100}"
for r in $(seq $ROUNDS); do
  for w in "${WL[@]}"; do
    for v in "$@"; do
      name=${v%%=*}; val=${v#*=}
      if [ -n "$val" ]; then export RTC_DEBUG="$val"; else unset RTC_DEBUG; fi
      timeout -k 10 240 python bench.py $w --mode frames --ab --no-cpu-baseline > gpurun_out/abk_$name.log 2>&1 || { echo "$name failed ($w)"; tail -5 gpurun_out/abk_$name.log; exit 1; }
      python - "$name" "$r" <<'PY'
import json, sys
d = [json.loads(l) for l in open(f"gpurun_out/abk_{sys.argv[1]}.log") if l.startswith("{")][-1]
print(json.dumps({"variant": sys.argv[1], "round": int(sys.argv[2]), "workload": d["config"]["workload"],
                  "gray_s": round(d["value"] / 1e3, 2), "ms_per_step": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "cold_kernel_ms": d.get("cold_kernel_ms"),
                  "jit_used": d.get("jit_used")}), flush=True)
PY
    done
  done
done
unset RTC_DEBUG
