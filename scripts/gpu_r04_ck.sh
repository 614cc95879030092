#!/bin/bash
# Round-4 A/B: more preloaded arbiter-cache entries -- 5v5 12 or 10 (variants "ckl12", "ckl10")
# against 8, 2v2 8 (variant "cks8") against 6; instance matrix + v1 parity on each variant.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_ck_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_ck_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
B5="$B --players 5 --steps 1200"
T="python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread"
FUTBOL_LIB_VARIANT=ckl12 step suite_ckl12 400 $T
FUTBOL_LIB_VARIANT=ckl10 step suite_ckl10 400 $T
FUTBOL_LIB_VARIANT=cks8 step suite_cks8 400 $T
for r in a b c; do
    step p5_$r 200 $B5
    FUTBOL_LIB_VARIANT=ckl12 step k12_$r 200 $B5
    FUTBOL_LIB_VARIANT=ckl10 step k10_$r 200 $B5
    step p2_$r 200 $B
    FUTBOL_LIB_VARIANT=cks8 step s8_$r 200 $B
done
