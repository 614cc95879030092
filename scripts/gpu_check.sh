# smoke, the -m gpu suite and bench lines (run via gpurun from the repo root)
#   OUT_DIR=name  PYTEST_K="expr" (pytest -k)  PYTEST_ARGS=...  BENCH="default v0 5v5"  (which bench lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_DIR:-check}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1 || { echo pytest failed; exit 1; }
fi
for b in ${BENCH:-default}; do
  case $b in
    default) args="" ;;
    k20) args="--steps 20 --warmup 5" ;;
    v0) args="--kind v0" ;;
    5v5) args="--players 5 --steps 1200" ;;
    r100) args="--rollout 100" ;;
    v0r) args="--kind v0 --rollout 100" ;;
    5v5r) args="--players 5 --steps 1200 --rollout 100" ;;
    *) args="$b" ;;
  esac
  timeout -k 10 300 python bench.py $args > $O/bench_$b.log 2>&1 || { echo bench $b failed; exit 1; }
done
echo rc=0
