set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STUDY_VARIANTS="default old cubes flat8 flat32" timeout -k 10 400 python tests/study_f32_error.py refraction reflect_refract cover table shadow_puppets cylinders three_sphere_scene metal > gpurun_out/r06_offset_study.jsonl 2> gpurun_out/r06_offset_study.err; echo "study rc=$?"
timeout -k 10 300 python scripts/graph_probe.py 15 > gpurun_out/r06_graph_probe.jsonl 2> gpurun_out/r06_graph_probe.err; echo "probe rc=$?"; cat gpurun_out/r06_graph_probe.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; echo "tests rc=$?"; tail -30 gpurun_out/pytest_gpu.log
