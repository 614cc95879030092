#!/bin/bash
# Round-4: the GPU suite on the product (LDS record slots 5 / 4 / 4 for N = 8 / 9 / 10), then
# N = 8 and 9 against the previous slot counts (variant "k89old": 4 / 3), and the 10v10 line.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_k89_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_k89_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
step suite_k89 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread
step p_8 200 $B --players 8 --steps 600
FUTBOL_LIB_VARIANT=k89old step o_8 200 $B --players 8 --steps 600
step p_9 200 $B --players 9 --steps 600
FUTBOL_LIB_VARIANT=k89old step o_9 200 $B --players 9 --steps 600
step p_10v10 200 $B --players 10 --steps 600
step p_8_b 200 $B --players 8 --steps 600
FUTBOL_LIB_VARIANT=k89old step o_8_b 200 $B --players 8 --steps 600
