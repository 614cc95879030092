#!/bin/bash
# Round-4 A/B: observation rows stored per wave through LDS (product) against per-lane element
# stores (variant "obsold", -DFUTBOL_OBS_LDS=0); the GPU suite on the product build first.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_obs_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_obs_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
step suite_obs 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread
step n_2v2_a 200 $B
FUTBOL_LIB_VARIANT=obsold step o_2v2_a 200 $B
step n_2v2_b 200 $B
FUTBOL_LIB_VARIANT=obsold step o_2v2_b 200 $B
step n_v0 200 $B --kind v0
FUTBOL_LIB_VARIANT=obsold step o_v0 200 $B --kind v0
step n_5v5 200 $B --players 5 --steps 1200
FUTBOL_LIB_VARIANT=obsold step o_5v5 200 $B --players 5 --steps 1200
step n_10v10 200 $B --players 10 --steps 600
FUTBOL_LIB_VARIANT=obsold step o_10v10 200 $B --players 10 --steps 600
step n_v0_b 200 $B --kind v0
FUTBOL_LIB_VARIANT=obsold step o_v0_b 200 $B --kind v0
