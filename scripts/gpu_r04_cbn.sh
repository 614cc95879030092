#!/bin/bash
# Round-4 A/B: arbiter-cache entries past the preloaded ones read 4 per batch (variant "cbn4") against
# 1 per batch (product) for 5v5 and 10v10, plus the GPU instance matrix on the variant.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_cbn_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_cbn_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
FUTBOL_LIB_VARIANT=cbn4 step suite_cbn4 600 python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread
step p_5v5 200 $B --players 5 --steps 1200
FUTBOL_LIB_VARIANT=cbn4 step c_5v5 200 $B --players 5 --steps 1200
step p_10v10 200 $B --players 10 --steps 600
FUTBOL_LIB_VARIANT=cbn4 step c_10v10 200 $B --players 10 --steps 600
step p_5v5_b 200 $B --players 5 --steps 1200
FUTBOL_LIB_VARIANT=cbn4 step c_5v5_b 200 $B --players 5 --steps 1200
step p_10v10_b 200 $B --players 10 --steps 600
FUTBOL_LIB_VARIANT=cbn4 step c_10v10_b 200 $B --players 10 --steps 600
