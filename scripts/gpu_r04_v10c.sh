#!/bin/bash
# Round-4 A/B, third set, over the product with 4 spill records in registers for N >= 6: cache
# batches of 8 (variant "cbn8", N >= 5) and the v_bias loads after the action phase for N >= 6
# (variant "lateb"); full GPU suite on the product, instance matrix + v1 parity on the variants.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_v10c_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_v10c_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line --players 10 --steps 600"
B5="python bench.py --no-cpu-baseline --no-rollout-line --players 5 --steps 1200"
T="python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread"
step suite_prod 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread
FUTBOL_LIB_VARIANT=cbn8 step suite_cbn8 400 $T
FUTBOL_LIB_VARIANT=lateb step suite_lateb 400 $T
for r in a b c; do
    step p_$r 200 $B
    FUTBOL_LIB_VARIANT=cbn8 step cbn8_$r 200 $B
    FUTBOL_LIB_VARIANT=lateb step lateb_$r 200 $B
    step p5_$r 200 $B5
    FUTBOL_LIB_VARIANT=cbn8 step cbn8_5_$r 200 $B5
done
