set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_v1_parity.py -x -q > gpurun_out/pytest_epw32.log 2>&1 && \
FUTBOL_EPW=16 timeout -k 10 600 python -m pytest tests/test_gpu_v1_parity.py -x -q -k "free_running or crowded" > gpurun_out/pytest_epw16.log 2>&1 && \
for E in 64 32 16; do FUTBOL_EPW=$E timeout -k 10 120 python bench.py --steps 3000 --no-cpu-baseline > gpurun_out/bench_e$E.log 2>&1 || exit 1; done && \
for E in 64 32 16; do FUTBOL_EPW=$E timeout -k 10 120 python bench.py --stamps --warmup 100 --steps 190 --profile-steps 10 > gpurun_out/stamps_e$E.log 2>&1 || exit 1; done
