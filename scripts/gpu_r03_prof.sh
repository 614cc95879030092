# round-3 end artifacts (part 2): rocprofv3 passes of the 5v5 (C5) and v0 (C3) step kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final3
mkdir -p $O
PROF_DIR=prof5 BENCH_ARGS="--players 5" STEPS=120 bash scripts/gpu_profile.sh > $O/profile5.log 2>&1 && \
PROF_DIR=prof0 BENCH_ARGS="--kind v0" bash scripts/gpu_profile.sh > $O/profile0.log 2>&1
echo rc=$?
