# quick loop: v1 parity tests + 2v2 / 5v5 bench lines (no cpu baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_v1_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_v1.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_q2.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --players 5 > gpurun_out/bench_q5.log 2>&1
