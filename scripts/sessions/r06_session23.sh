set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" "jit_flags=-DRTC_EXP_CUT_DEPTH=6" "jit_flags=-DRTC_EXP_CUT_DEPTH=5" "jit_flags=-DRTC_EXP_CUT_DEPTH=4" "jit_flags=-DRTC_EXP_CUT_DEPTH=3" "jit_flags=-DRTC_EXP_CUT_DEPTH=2" ""; do
  RTC_DEBUG="$v" timeout -k 10 240 python scripts/cut_depth_probe.py cover table >> gpurun_out/r06_cut_depth.jsonl 2> gpurun_out/r06_cut_depth.err || { tail -5 gpurun_out/r06_cut_depth.err; exit 1; }
done
cat gpurun_out/r06_cut_depth.jsonl
