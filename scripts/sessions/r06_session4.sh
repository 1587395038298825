set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python scripts/parity_report.py --sizes 160x120,320x200 --out gpurun_out/r06_parity_small.json > gpurun_out/r06_parity_small.log 2>&1; echo "parity small rc=$?"
timeout -k 10 500 python scripts/parity_report.py --configs --out gpurun_out/r06_parity_configs.json > gpurun_out/r06_parity_configs.log 2>&1; echo "parity configs rc=$?"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
ROUNDS=3 bash scripts/ab_jit_flags.sh "--steps 1000 --mode frames --ab --no-cpu-baseline" "base=" "hoist=-DRTC_DIRECT_HOIST=1" > gpurun_out/r06_ab_hoist.jsonl 2>&1; echo "ab hoist rc=$?"; cat gpurun_out/r06_ab_hoist.jsonl
for i in 1 2; do for st in null side; do timeout -k 10 240 python bench.py --steps 20 --warmup 5 --mode frames --ab --no-cpu-baseline --stream $st > gpurun_out/r06_stream_$st.log 2>&1 || exit 1; python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r06_stream_$st.log') if l.startswith('{')][-1]; print('$st', round(d['value']/1e3,1), d['ms_per_step'], d['roofline']['kernel_ms'])"; done; done
bash scripts/shard_pmc.sh > gpurun_out/r06_shard_pmc.log 2>&1; echo "shard pmc rc=$?"; cat gpurun_out/r06_shard_pmc.log | cut -c1-300
