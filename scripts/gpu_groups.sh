# A/B of the async env-group count in bench.py (v1 2v2, no cpu baseline), then the v1 parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_v1_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_v1.log 2>&1 && \
for g in 1 2 4 8; do timeout -k 10 300 python bench.py --no-cpu-baseline --groups $g > gpurun_out/bench_g$g.log 2>&1 || exit 1; done
