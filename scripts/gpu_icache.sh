# instruction-cache counters (SQC_ICACHE_*, SQ_IFETCH; one --pmc pass of <= 8 SQ counters) for the step
# kernels of the C2 (2v2), C5 (5v5) and C3 (v0) benches; run via gpurun from the repo root
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${PROF_DIR:-icache}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for cfg in "c2:" "c5:--players 5" "c3:--kind v0"; do
  t=${cfg%%:*}; a=${cfg#*:}
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/$t -o run --output-format csv -- python3 $R/bench.py --steps 300 --warmup 20 \
      --no-cpu-baseline --no-rollout-line --profile-steps 20 --graph 0 $a > $OUT/$t.log 2>&1 || { echo "pass $t failed"; exit 1; }
done
echo icache rc=0
