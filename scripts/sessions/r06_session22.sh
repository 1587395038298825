set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_knobs.sh "probe=" "noprobe=cold_probe=0" > gpurun_out/r06_ab_probe.jsonl 2>&1 || { tail -5 gpurun_out/r06_ab_probe.jsonl; exit 1; }
cat gpurun_out/r06_ab_probe.jsonl | cut -c1-220
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t22.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06_t22.log
