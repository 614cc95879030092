#!/bin/bash
# Round-4: full GPU suite on the product (late v_bias for N >= 6, cache batches of 8), the 10v10
# line, and the 5v5 A/B of the late v_bias load (variant "lateb5", N >= 5).
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_l5_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_l5_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line --players 10 --steps 600"
B5="python bench.py --no-cpu-baseline --no-rollout-line --players 5 --steps 1200"
T="python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread"
step suite_prod 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread
FUTBOL_LIB_VARIANT=lateb5 step suite_lateb5 400 $T
step p10_a 200 $B
step p10_b 200 $B
for r in a b c; do
    step p5_$r 200 $B5
    FUTBOL_LIB_VARIANT=lateb5 step l5_$r 200 $B5
done
