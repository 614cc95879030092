#!/bin/bash
# Round-4 5v5 A/B: 4 or 2 preloaded arbiter-cache entries (variants "ckl4", "ckl2") against 8
# (product) now that the entries past them are read 8 per batch; instance matrix + v1 parity on each.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_ckl_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_ckl_steps.txt
        exit 1
    fi
}
B5="python bench.py --no-cpu-baseline --no-rollout-line --players 5 --steps 1200"
T="python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread"
FUTBOL_LIB_VARIANT=ckl4 step suite_ckl4 400 $T
FUTBOL_LIB_VARIANT=ckl2 step suite_ckl2 400 $T
for r in a b c; do
    step p5_$r 200 $B5
    FUTBOL_LIB_VARIANT=ckl4 step k4_$r 200 $B5
    FUTBOL_LIB_VARIANT=ckl2 step k2_$r 200 $B5
done
