# bench value vs K with and without staggered episode phases
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${ST_OUT:-stagger}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_v1_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_v1.log 2>&1 || { echo parity-failed; exit 1; }
for st in 1 0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --stagger $st --steps 20 --warmup 5 > $O/bench_s${st}_k20.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --stagger $st --steps 1200 > $O/bench_s${st}_k1200.log 2>&1 || exit 1
done
echo stagger-ok
