#!/bin/bash
# Round-4 rocprofv3 profile of the 10v10 step kernel (kernel trace + stats, SQ counters, PMC traffic).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PROF_DIR=prof_10v10 STEPS=120 BENCH_ARGS="--players 10 --steps 600" bash scripts/gpu_profile.sh > gpurun_out/prof_10v10.log 2>&1 && grep -q "profile rc=0" gpurun_out/prof_10v10.log
echo "r04 prof10 rc=$?"
