# GPU parity (all -m gpu tests) + the driver's bench invocations
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${B2_OUT:-b2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo gpu-tests-failed; tail -20 $O/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --players 5 --no-cpu-baseline > $O/bench_5v5.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --kind v0 --no-cpu-baseline > $O/bench_v0.log 2>&1 || exit 1
echo b2-ok
