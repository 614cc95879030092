# round-3 end artifacts (part 3): the C3 bench line and v0 rocprofv3 passes after the v0 pair layout
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 300 python bench.py --kind v0 > $O/bench_v0.log 2>&1 && \
PROF_DIR=prof0 BENCH_ARGS="--kind v0" bash scripts/gpu_profile.sh > $O/profile0.log 2>&1
echo rc=$?
