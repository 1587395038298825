# shared helper: run LABEL CMD... -> one summary line from bench's JSON
run() {
  local label=$1; shift
  local line
  line=$(timeout -k 10 120 "$@" 2>/dev/null | grep '^{')
  echo "$label :: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("value=%.0f Mray/s kernel_ms=%.4f frac=%.4f rays/frame=%d" % (d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["config"]["rays_per_frame"]))' 2>&1)" | tee -a gpurun_out/ab.log
}
