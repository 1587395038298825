#!/bin/bash
# One gpurun session, steps chosen by name (each with its own time limit; a
# crash or timeout, rc other than 0/1, ends the session):
#   tests    pytest -m gpu (whole suite)            -> gpurun_out/pytest_gpu.log
#   bctests  the same suite on the RTC_BOUNDS_CHECK build (_lib_bc)
#   smoke    __graft_entry__.smoke()
#   bench    bench.py with the driver's flags, then 1000 steps; f64 line
#   pool     bench lines of the pool configs (reflect_refract, cover/table 4K)
#   initprobe  start-up step timings of a bare HIP process      -> gpurun_out/initprobe.log
#   shards   per-shard kernel times (scripts/shard_times.py)  -> gpurun_out/shards.log
#   shardtail  item log of one 8-way shard at split 8 and 16 -> gpurun_out/shardtail.log
#   profset  the round's profile set (scripts/profile_round.sh)  -> gpurun_out/r04_*
#   prof     rocprofv3 --kernel-trace --stats of the bench     -> gpurun_out/prof_*
# Usage: scripts/gpu_session.sh tests smoke bench ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/ray-tracer-challenge-rs_amd/rtc_amd
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; ok $rc || exit $rc ;;
    bctests)
      RTC_LIBRARY=$L/_lib_bc/librtc.so RTC_JIT_CACHE=0 timeout -k 10 600 python -u -m pytest tests -m gpu -q \
        --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_bc.log 2>&1
      rc=$?; echo "bctests rc=$rc"; tail -15 gpurun_out/pytest_gpu_bc.log; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok $rc || exit $rc ;;
    bench)
      timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1
      rc=$?; echo "bench(driver flags) rc=$rc"; tail -c 3000 gpurun_out/bench_driver.log; echo; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/bench_1000.log 2>&1
      rc=$?; echo "bench(1000) rc=$rc"; tail -c 1500 gpurun_out/bench_1000.log; echo; [ $rc -eq 0 ] || exit $rc ;;
    pool)
      : > gpurun_out/bench_pool.log
      for a in "--scene reflect_refract" "--scene cover --width 3840 --height 2160 --steps 300" \
               "--scene table --width 3840 --height 2160 --steps 300"; do
        timeout -k 10 240 python bench.py $a --no-cpu-baseline >> gpurun_out/bench_pool.log 2>&1
        rc=$?; echo "pool $a rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done
      tail -c 2000 gpurun_out/bench_pool.log; echo ;;
    ab)  # this tree's build against the builds in AB_VARIANTS (rtc_amd/_lib_*), alternating, 2 rounds
      : > gpurun_out/ab.log
      for r in $(seq ${AB_ROUNDS:-2}); do
        for v in _lib ${AB_VARIANTS:-_lib_acc64}; do
          # AB_ONLY=direct: three_sphere only (the direct kernel)
          if [ "${AB_ONLY:-}" = direct ]; then set -- "--scene three_sphere_scene --steps 1000"; else
            set -- "--scene three_sphere_scene" "--scene reflect_refract" "--scene cover --width 3840 --height 2160 --steps 300" \
                   "--scene table --width 3840 --height 2160 --steps 300"; fi
          for a in "$@"; do
            out=$(RTC_LIBRARY=$L/$v/librtc.so timeout -k 10 200 python bench.py $a --no-cpu-baseline --ab 2>>gpurun_out/ab.log | grep '^{')
            rc=$?; [ $rc -eq 0 ] || { echo "ab $v $a rc=$rc"; exit 1; }
            echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['config']['workload'], 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'cold', d.get('cold_kernel_ms'), 'jit', d.get('jit_used'))" | tee -a gpurun_out/ab.log
          done
        done
      done ;;
    abenv)  # environment knobs on this build (scripts/ab_env.sh): AB_SCENES, AB_ENVS (space-separated, X=0 = default)
      timeout -k 10 1000 bash scripts/ab_env.sh "${AB_SCENES:-reflect_refract}" ${AB_ENVS:-X=0} > gpurun_out/abenv.log 2>&1
      rc=$?; echo "abenv rc=$rc"; cat gpurun_out/abenv.log; [ $rc -eq 0 ] || exit $rc ;;
    coldtail)  # item logs of a cold and a warm launch (scripts/cold_tail.py)
      : > gpurun_out/coldtail.log
      for a in "reflect_refract 1920 1080" "cover 3840 2160"; do
        timeout -k 10 200 python scripts/cold_tail.py $a >> gpurun_out/coldtail.log 2>&1
        rc=$?; [ $rc -eq 0 ] || { echo "coldtail rc=$rc"; tail -5 gpurun_out/coldtail.log; exit $rc; }
      done
      grep -v amdgpu.ids gpurun_out/coldtail.log | cut -c1-2500 ;;
    partest)  # one test file (PARTEST, default the parity tests)
      timeout -k 10 600 python -u -m pytest ${PARTEST:-tests/test_gpu_parity.py} -m gpu -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/partest.log 2>&1
      rc=$?; echo "partest rc=$rc"; tail -15 gpurun_out/partest.log; ok $rc || exit $rc ;;
    jitdump)  # per-scene headers of the bench scenes for scripts/jit_isa.sh
      mkdir -p gpurun_out/jit
      for a in "--scene three_sphere_scene" "--scene reflect_refract" "--scene cover --width 3840 --height 2160" \
               "--scene table --width 3840 --height 2160"; do
        RTC_DEBUG=jit_dump=gpurun_out/jit RTC_JIT_CACHE=0 timeout -k 10 200 python bench.py $a --steps 20 --no-cpu-baseline \
          > /dev/null 2>>gpurun_out/jitdump.log || { echo "jitdump $a failed"; exit 1; }
      done
      ls gpurun_out/jit ;;
    oneshot)  # where a one-shot render's time goes (RTC_DEBUG=trace_init steps), torch-free child, twice
      for i in 1 2; do
        RTC_DEBUG=trace_init=1 timeout -k 10 120 python bench.py --one-shot-child > gpurun_out/oneshot_$i.log 2>&1
        rc=$?; echo "oneshot rc=$rc"; grep -v amdgpu.ids gpurun_out/oneshot_$i.log; [ $rc -eq 0 ] || exit $rc
      done ;;
    initprobe)  # start-up steps of a bare HIP process (scripts/init_probe.cpp), with and without RCCL loaded
      : > gpurun_out/initprobe.log
      for a in ${PROBES:-"" "rccl" "" "rccl" "prefault=touch" "prefault=huge" "prefault=threads" "prefault=small" "prefault=register"}; do
        timeout -k 10 60 scripts/_init_probe $a >> gpurun_out/initprobe.log 2>&1
        rc=$?; [ $rc -eq 0 ] || { echo "initprobe $a rc=$rc"; exit $rc; }
      done
      cat gpurun_out/initprobe.log ;;
    shards)  # per-shard kernel time at N = 1 and 8 (what each rank renders), cover and table 4K;
             # SHARD_ENVS: environment settings to sweep ("-" = none)
      : > gpurun_out/shards.log
      for e in ${SHARD_ENVS:--}; do
        for sc in cover table; do
          [ "$e" = - ] || echo "$e" >> gpurun_out/shards.log
          env ${e/#-/} SHARD_COUNTS=${SHARD_COUNTS:-1,8} timeout -k 10 300 python scripts/shard_times.py $sc 3840 2160 >> gpurun_out/shards.log 2>&1
          rc=$?; [ $rc -eq 0 ] || { echo "shards $sc rc=$rc"; tail -5 gpurun_out/shards.log; exit $rc; }
        done
      done
      grep -v amdgpu.ids gpurun_out/shards.log ;;
    shardtail)  # item log of shard 0 of 8 (cover 4K) at split 8 and 16
      : > gpurun_out/shardtail.log
      for sm in 3 4; do
        RTC_DEBUG=split_max=$sm timeout -k 10 300 python scripts/shard_tail.py cover 3840 2160 8 0 >> gpurun_out/shardtail.log 2>&1
        rc=$?; [ $rc -eq 0 ] || { echo "shardtail rc=$rc"; tail -5 gpurun_out/shardtail.log; exit $rc; }
      done
      grep -v amdgpu.ids gpurun_out/shardtail.log | cut -c1-1500 ;;
    roundbench)  # the round's bench lines (scripts/round_bench.sh; ROUND, default r04)
      ROUND=${ROUND:-r04} timeout -k 10 1000 bash scripts/round_bench.sh > gpurun_out/roundbench.log 2>&1
      rc=$?; echo "roundbench rc=$rc"; cat gpurun_out/roundbench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc ;;
    profset)  # the round's profile set (scripts/profile_round.sh; ROUND, default r04)
      ROUND=${ROUND:-r04} bash scripts/profile_round.sh > gpurun_out/profset.log 2>&1
      rc=$?; echo "profset rc=$rc"; grep -v amdgpu.ids gpurun_out/profset.log | cut -c1-400 | tail -40; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      for sc in three_sphere_scene reflect_refract; do
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$sc -o run -- \
          python3 bench.py --scene $sc --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/prof_$sc.log 2>&1
        rc=$?; echo "prof $sc rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
