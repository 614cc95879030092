#!/bin/bash
# Round-4 10v10 A/B, second set: 4 spill records in registers (variant "sr4") and cache batches of 8
# (variant "cbn8", N >= 5) against the product (2 spill records, batches of 4); instance matrix +
# v1 parity on each variant, 5v5 for cbn8.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_v10b_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_v10b_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line --players 10 --steps 600"
B5="python bench.py --no-cpu-baseline --no-rollout-line --players 5 --steps 1200"
T="python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread"
FUTBOL_LIB_VARIANT=sr4 step suite_sr4 400 $T
FUTBOL_LIB_VARIANT=cbn8 step suite_cbn8 400 $T
step p_a 200 $B
FUTBOL_LIB_VARIANT=sr4 step sr4_a 200 $B
FUTBOL_LIB_VARIANT=cbn8 step cbn8_a 200 $B
step p_b 200 $B
FUTBOL_LIB_VARIANT=sr4 step sr4_b 200 $B
FUTBOL_LIB_VARIANT=cbn8 step cbn8_b 200 $B
step p5_a 200 $B5
FUTBOL_LIB_VARIANT=cbn8 step cbn8_5_a 200 $B5
