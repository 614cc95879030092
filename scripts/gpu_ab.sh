# A/B bench lines of library variants (run via gpurun from the repo root):
#   AB="head: main:" (variant:extra-bench-args ... ; "main" = libfutbol_amd.so)  OUT_DIR=name  PYTEST_K=expr
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_DIR:-ab}
mkdir -p $O
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "$PYTEST_K" > $O/pytest.log 2>&1 || { echo pytest failed; exit 1; }
fi
i=0
for spec in $AB; do
  v=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
  i=$((i+1))
  if [ "$v" = main ]; then lv=""; else lv=$v; fi
  FUTBOL_LIB_VARIANT=$lv timeout -k 10 300 python bench.py --no-cpu-baseline --no-rollout-line $args > $O/b${i}_$v.log 2>&1 || { echo bench $spec failed; exit 1; }
  echo "$spec $(grep -o '"value": [0-9.e+]*' $O/b${i}_$v.log) $(grep -o '"kernel_ms": [0-9.e+-]*' $O/b${i}_$v.log)"
done
echo rc=0
