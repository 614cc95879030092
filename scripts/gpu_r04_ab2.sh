#!/bin/bash
# Round-4 A/B: LLVM's pre-RA exec-mask optimization on (variant "prera", ISA-gated) against the product,
# and the driver's short timed region (K = 20) replayed from a hipGraph vs launched one by one.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_ab2_steps.txt
    if [ $rc -ge 2 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_ab2_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
step p_2v2_a 200 $B
FUTBOL_LIB_VARIANT=prera step v_2v2_a 200 $B
step p_2v2_b 200 $B
FUTBOL_LIB_VARIANT=prera step v_2v2_b 200 $B
step p_v0 200 $B --kind v0
FUTBOL_LIB_VARIANT=prera step v_v0 200 $B --kind v0
step p_5v5 200 $B --players 5 --steps 1200
FUTBOL_LIB_VARIANT=prera step v_5v5 200 $B --players 5 --steps 1200
FUTBOL_BENCH_DEBUG=1 step k20_graph_a 200 $B --steps 20 --warmup 5
FUTBOL_BENCH_DEBUG=1 step k20_direct_a 200 $B --steps 20 --warmup 5 --direct 1
FUTBOL_BENCH_DEBUG=1 step k20_graph_b 200 $B --steps 20 --warmup 5
FUTBOL_BENCH_DEBUG=1 step k20_direct_b 200 $B --steps 20 --warmup 5 --direct 1
FUTBOL_BENCH_DEBUG=1 step k300_direct 200 $B --steps 300 --direct 1
FUTBOL_LIB_VARIANT=prera step v_suite 500 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread
