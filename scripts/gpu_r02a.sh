set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
O=gpurun_out/r02a
hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_fp64 scripts/ubench_fp64.hip && \
timeout -k 10 120 /tmp/ubench_fp64 > $O/ubench.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_k20.log 2>&1
echo rc=$?
