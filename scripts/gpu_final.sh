# round-end validation: smoke, the whole -m gpu suite, the bench line (default and the driver's
# short K), C3 / C5 lines, the 2-rank rehearsal, then the rocprofv3 passes of the 2v2 and 5v5 bench kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 && \
timeout -k 10 300 python bench.py --kind v0 > $O/bench_v0.log 2>&1 && \
timeout -k 10 300 python bench.py --players 5 --steps 1200 > $O/bench_5v5.log 2>&1 && \
bash scripts/gpu_multirank.sh && cp gpurun_out/bench_2rank.log $O/ && \
bash scripts/gpu_profile.sh > $O/profile.log 2>&1 && \
PROF_DIR=prof5 BENCH_ARGS="--players 5" STEPS=120 bash scripts/gpu_profile.sh > $O/profile5.log 2>&1
echo rc=$?
