# kernel trace + stats of the default bench command (no counters)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/trace
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/bench.py ${BENCH_ARGS:-} > $OUT/trace.log 2>&1
