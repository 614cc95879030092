# round-3 end artifacts (part 1): smoke, bench lines (C2 default and the driver's short line, C3, C5), 2v2 rocprofv3 passes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && \
timeout -k 10 300 python bench.py --kind v0 > $O/bench_v0.log 2>&1 && \
timeout -k 10 300 python bench.py --players 5 --steps 1200 > $O/bench_5v5.log 2>&1 && \
PROF_DIR=prof bash scripts/gpu_profile.sh > $O/profile.log 2>&1
echo rc=$?
