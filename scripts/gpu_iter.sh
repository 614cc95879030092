# iteration loop on one box: v1 parity tests, 2v2 + 5v5 bench lines, stamps of 2v2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${IT_OUT:-iter}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_v1_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_v1.log 2>&1 || { echo "parity failed"; tail -30 $O/pytest_v1.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${IT_STEPS:-1200} > $O/bench2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${IT_STEPS:-1200} --players 5 > $O/bench5.log 2>&1 || exit 1
if [ -n "$IT_STAMPS" ]; then
  timeout -k 10 300 python bench.py --stamps --warmup 40 --steps 300 --profile-steps 10 --snapshots 64 > $O/stamps.log 2>&1 || exit 1
fi
echo iter-ok
