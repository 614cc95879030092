# the whole -m gpu suite, then A/B bench lines (scripts/gpu_ab.sh specs in AB)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_DIR:-suite_ab}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.log 2>&1 || { echo pytest failed; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
OUT_DIR=${OUT_DIR:-suite_ab} bash scripts/gpu_ab.sh
