# smoke, the -m gpu suite and the C2 bench line (run via gpurun from the repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_DIR:-check}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
echo rc=$?
