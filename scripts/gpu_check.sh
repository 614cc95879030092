set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3000 > gpurun_out/bench.log 2>&1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --stamps --warmup 100 --steps 190 --profile-steps 10 > gpurun_out/stamps.log 2>&1
