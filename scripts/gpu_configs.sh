# bench + rocprofv3 passes for the other single-GPU configs (C3 v0 hard-coded opponent, C5 5v5)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --kind v0 > gpurun_out/bench_v0.log 2>&1 && \
timeout -k 10 300 python bench.py --players 5 > gpurun_out/bench_5v5.log 2>&1 && \
timeout -k 10 300 python bench.py --players 10 --no-cpu-baseline > gpurun_out/bench_10v10.log 2>&1 && \
BENCH_ARGS="--kind v0" bash scripts/gpu_profile.sh > gpurun_out/profile_v0.log 2>&1 && mv gpurun_out/prof gpurun_out/prof_v0 && \
BENCH_ARGS="--players 5" bash scripts/gpu_profile.sh > gpurun_out/profile_5v5.log 2>&1 && mv gpurun_out/prof gpurun_out/prof_5v5
