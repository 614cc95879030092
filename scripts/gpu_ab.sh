# A/B timing of library variants in one box: VARIANTS="old ''" (empty = the default library)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/${AB_OUT:-ab}.log; : > $OUT
for rep in 1 2; do
  for v in ${VARIANTS:-old default}; do
    vv=$v; [ "$v" = default ] && vv=""
    FUTBOL_LIB_VARIANT=$vv timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1500 ${BENCH_ARGS:-} > gpurun_out/ab_one.log 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/ab_one.log)" >> $OUT
  done
done
