# iterate: v1 parity tests, then the bench (no cpu baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/it
timeout -k 10 600 python -u -m pytest tests/test_gpu_v1_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/it/pytest_v1.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/it/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1200 --players 5 > gpurun_out/it/bench5.log 2>&1
echo rc=$?
