# smoke + GPU parity tests + bench (+ optional rocprofv3 passes), via gpurun from the repo root
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
if [ -n "$PROFILE" ]; then bash scripts/gpu_profile.sh > gpurun_out/profile.log 2>&1; fi
