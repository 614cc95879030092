# iterate: v1 parity tests, then the bench (no cpu baseline); STAMPS=1 adds the tail study
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/it
timeout -k 10 600 python -u -m pytest tests/test_gpu_v1_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/it/pytest_v1.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/it/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1200 --players 5 > gpurun_out/it/bench5.log 2>&1 && \
if [ -n "$STAMPS" ]; then timeout -k 10 300 python bench.py --stamps --warmup 150 --steps 100 --profile-steps 10 --snapshots 60 --snapshot-stride 3 --stamps-dump gpurun_out/it/waves.npy > gpurun_out/it/stamps.log 2>&1; fi
echo rc=$?
