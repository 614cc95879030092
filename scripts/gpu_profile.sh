# rocprofv3 passes for the bench's dominant kernel (run via gpurun from the repo root).
#   kernel trace + stats, SQ instruction/cycle counters, FETCH_SIZE, WRITE_SIZE (separate
#   --pmc passes, never combined with sys/runtime tracing), plus the same FETCH/WRITE passes
#   over scripts/pmc_calib.hip to correct the counters for our access widths.
# Then: python scripts/pmc_traffic.py --prof gpurun_out/prof --round rNN  (CPU side)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${PROF_DIR:-prof}
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -o $OUT/pmc_calib $R/scripts/pmc_calib.hip || exit 1
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline --no-rollout-line --profile-steps 20 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-rollout-line ${BENCH_ARGS:-} > $OUT/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/sq -o run --output-format csv -- python3 $B --graph 0 > $OUT/sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $B --graph 0 > $OUT/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $B --graph 0 > $OUT/write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 $B --graph 0 > $OUT/sq2.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib_fetch -o run --output-format csv -- $OUT/pmc_calib > $OUT/calib_fetch.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/calib_write -o run --output-format csv -- $OUT/pmc_calib > $OUT/calib_write.log 2>&1
echo "profile rc=$?"
