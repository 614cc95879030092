#!/bin/bash
# Round-4 5v5 A/B: 6 spill records in registers (variant "kx6") against 4 (product).
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_kx6_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_kx6_steps.txt
        exit 1
    fi
}
T="python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread"
B5="python bench.py --no-cpu-baseline --no-rollout-line --players 5 --steps 1200"
FUTBOL_LIB_VARIANT=kx6 step suite_kx6 400 $T
for r in a b c; do
    step p5_$r 200 $B5
    FUTBOL_LIB_VARIANT=kx6 step x6_$r 200 $B5
done
