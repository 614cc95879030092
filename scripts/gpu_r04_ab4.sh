#!/bin/bash
# Round-4 A/B: the exact squares' slow path as one wave work list (product) against per-lane rounds
# (variant "nowl"); the GPU suite on the product build.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_ab4_steps.txt
    if [ $rc -ge 2 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_ab4_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
step suite4 500 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread
step w_2v2_a 200 $B
FUTBOL_LIB_VARIANT=nowl step x_2v2_a 200 $B
step w_2v2_b 200 $B
FUTBOL_LIB_VARIANT=nowl step x_2v2_b 200 $B
step w_5v5 200 $B --players 5 --steps 1200
FUTBOL_LIB_VARIANT=nowl step x_5v5 200 $B --players 5 --steps 1200
step w_5v5_b 200 $B --players 5 --steps 1200
FUTBOL_LIB_VARIANT=nowl step x_5v5_b 200 $B --players 5 --steps 1200
