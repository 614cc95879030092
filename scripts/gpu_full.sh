# full GPU suite + 2v2 / 5v5 / v0 benches (no cpu baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/full/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1200 --players 5 > gpurun_out/full/bench5.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --kind v0 > gpurun_out/full/bench0.log 2>&1
echo rc=$?
