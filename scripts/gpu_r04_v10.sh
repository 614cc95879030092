#!/bin/bash
# Round-4 10v10 A/B: 4 preloaded arbiter-cache entries for N >= 6 (variant "ck4") and 2 spill
# records in registers (variant "sr2") against the product; instance matrix + v1 parity on each.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_v10_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_v10_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line --players 10 --steps 600"
T="python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread"
FUTBOL_LIB_VARIANT=ck4 step suite_ck4 400 $T
FUTBOL_LIB_VARIANT=sr2 step suite_sr2 400 $T
step p_a 200 $B
FUTBOL_LIB_VARIANT=ck4 step ck4_a 200 $B
FUTBOL_LIB_VARIANT=sr2 step sr2_a 200 $B
step p_b 200 $B
FUTBOL_LIB_VARIANT=ck4 step ck4_b 200 $B
FUTBOL_LIB_VARIANT=sr2 step sr2_b 200 $B
