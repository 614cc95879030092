# HEAD validation: smoke, the whole -m gpu suite, the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/head
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
echo rc=$?
