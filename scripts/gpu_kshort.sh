# the driver's short bench line (K = 20, W = 5) against longer timed regions
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ks
for k in 20 100 300; do timeout -k 10 300 python bench.py --no-cpu-baseline --steps $k --warmup 5 > gpurun_out/ks/k$k.log 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ks/driver.log 2>&1
echo rc=$?
