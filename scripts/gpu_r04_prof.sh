#!/bin/bash
# Round-4 profiles of the final kernels: scripts/gpu_profile.sh for C2 (2v2), C5 (5v5) and C3 (v0),
# then the bench lines (C2 with the CPU baseline and the rollout companion, the driver's short line).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PROF_DIR=prof_2v2 bash scripts/gpu_profile.sh > gpurun_out/prof_2v2.log 2>&1 && grep -q "profile rc=0" gpurun_out/prof_2v2.log && \
PROF_DIR=prof_5v5 BENCH_ARGS="--players 5" bash scripts/gpu_profile.sh > gpurun_out/prof_5v5.log 2>&1 && grep -q "profile rc=0" gpurun_out/prof_5v5.log && \
PROF_DIR=prof_v0 BENCH_ARGS="--kind v0" bash scripts/gpu_profile.sh > gpurun_out/prof_v0.log 2>&1 && grep -q "profile rc=0" gpurun_out/prof_v0.log && \
python scripts/pmc_traffic.py --prof gpurun_out/prof_2v2 --round r04 > gpurun_out/traffic_2v2.log 2>&1 && \
python scripts/pmc_traffic.py --prof gpurun_out/prof_5v5 --round r04 --players 5 > gpurun_out/traffic_5v5.log 2>&1 && \
python scripts/pmc_traffic.py --prof gpurun_out/prof_v0 --round r04 --kind v0 --players 2 > gpurun_out/traffic_v0.log 2>&1 && \
cp profiles/r04/traffic.json gpurun_out/traffic_r04.json && \
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/final_bench_k20.json 2>> gpurun_out/final_bench.err && \
timeout -k 10 200 python bench.py --kind v0 --no-cpu-baseline > gpurun_out/final_bench_v0.json 2>> gpurun_out/final_bench.err && \
timeout -k 10 200 python bench.py --players 5 --steps 1200 --no-cpu-baseline > gpurun_out/final_bench_5v5.json 2>> gpurun_out/final_bench.err && \
timeout -k 10 200 python bench.py --players 10 --steps 600 --no-cpu-baseline > gpurun_out/final_bench_10v10.json 2>> gpurun_out/final_bench.err
echo "r04 prof rc=$?"
