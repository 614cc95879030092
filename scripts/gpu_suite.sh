# the whole -m gpu suite (with the instance matrix), then bench lines of the head build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc: $(tail -1 $O/pytest_gpu.log)"
grep -o 'AssertionError: N=.*' $O/pytest_gpu.log | head -10
grep -E '^FAILED|illegal' $O/pytest_gpu.log | head -10
[ $rc -ne 0 ] && exit 1
[ -n "$AB" ] && OUT_DIR=suite bash scripts/gpu_ab.sh
echo done
