set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/sessions/r06_session40.sh || exit 1
WORKLOADS="--steps 20 --warmup 5" ROUNDS=3 bash scripts/ab_knobs.sh "base=" "o10=direct_oversub=10" "o25=direct_oversub=25" "o40=direct_oversub=40" > gpurun_out/r06_ab_oversub20.jsonl 2>&1 || { tail -3 gpurun_out/r06_ab_oversub20.jsonl; exit 1; }
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r06_ab_oversub20.jsonl"):
    if l.startswith("{"):
        r = json.loads(l); d[r["variant"]].append(r["gray_s"])
for k, v in d.items(): print(k, v)
PY
