# envs-per-wave A/B on one box (FUTBOL_EPW selects the v1 kernel instantiation)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/${AB_OUT:-epw}.log; : > $OUT
for rep in 1 2; do
  for e in ${EPWS:-64 32}; do
    FUTBOL_EPW=$e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1500 ${BENCH_ARGS:-} > gpurun_out/ab_one.log 2>&1 || exit 1
    echo "$e $(tail -1 gpurun_out/ab_one.log)" >> $OUT
  done
done
