# every step instance (tests/test_gpu_instances.py) for the head build and for variants, then A/B bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/inst
mkdir -p $O
for v in ${VARIANTS:-main}; do
  lv=$v; [ "$v" = main ] && lv=""
  FUTBOL_LIB_VARIANT=$lv timeout -k 10 400 python -u -m pytest tests/test_gpu_instances.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1
  rc=$?
  echo "$v: $(grep -c PASSED $O/pytest_$v.log) passed, $(grep -c FAILED $O/pytest_$v.log) failed (rc=$rc)"
  grep -o 'AssertionError: N=[^"]*' $O/pytest_$v.log | head -5
  case $rc in 124|134|137|139) echo "stopping after rc=$rc"; exit 1;; esac
done
[ -n "$AB" ] && OUT_DIR=inst bash scripts/gpu_ab.sh
echo done
