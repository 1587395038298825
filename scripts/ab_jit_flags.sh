#!/bin/bash
# Same-box A/B of per-scene build flags (RTC_DEBUG=jit_flags=..., which only
# the hipRTC builds see), alternating ROUNDS times:
#   scripts/ab_jit_flags.sh "<bench args>" "name=flags" "name=flags" ...
# ("base=" = no extra flags).  One JSON summary line per run.
set -u
ARGS=$1; shift
ROUNDS=${ROUNDS:-3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq $ROUNDS); do
  for v in "$@"; do
    name=${v%%=*}; flags=${v#*=}
    if [ -n "$flags" ]; then export RTC_DEBUG="jit_flags=$flags"; else unset RTC_DEBUG; fi
    timeout -k 10 240 python bench.py $ARGS > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/ab_$name.log; exit 1; }
    python - "$name" "$r" <<'PY'
import json, sys
d = [json.loads(l) for l in open(f"gpurun_out/ab_{sys.argv[1]}.log") if l.startswith("{")][-1]
print(json.dumps({"variant": sys.argv[1], "round": int(sys.argv[2]), "workload": d["config"]["workload"],
                  "gray_s": round(d["value"] / 1e3, 2), "ms_per_step": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "jit_used": d.get("jit_used"),
                  "sclk": (d.get("device_state") or {}).get("before", {}).get("sclk_mhz")}), flush=True)
PY
  done
done
unset RTC_DEBUG
