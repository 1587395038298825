set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STUDY_VARIANTS="default sph1e5 sph15e6 sph5e6 sph3e6" timeout -k 10 500 python tests/study_f32_error.py refraction reflect_refract cover table shadow_puppets cylinders three_sphere_scene metal > gpurun_out/r06_sphere_study.jsonl 2> gpurun_out/r06_sphere_study.err; echo "study rc=$?"
{ timeout -k 10 120 python scripts/shard_tail.py cover 3840 2160 1 0 && timeout -k 10 120 python scripts/shard_tail.py cover 3840 2160 8 0,3,7 && timeout -k 10 120 python scripts/shard_tail.py table 3840 2160 1 0 && timeout -k 10 120 python scripts/shard_tail.py table 3840 2160 8 0,5; } > gpurun_out/r06_shard_tail.jsonl 2> gpurun_out/r06_shard_tail.err; echo "tail rc=$?"
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_driver_$i.log 2>&1; echo "bench$i rc=$?"; done
