set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t35.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/r06_t35.log; grep -E "FAILED|^E " gpurun_out/r06_t35.log | head; tail -1 gpurun_out/r06_t35.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke35.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r06_smoke35.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench35.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r06_bench35.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e3,1), d['ms_per_step'], d['frame_latency_ms'], d['roofline']['frac'], {k: round(v['ms_per_step'],4) for k,v in d['tile_split'].items()})"; exit $rc
