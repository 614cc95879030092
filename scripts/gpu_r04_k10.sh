#!/bin/bash
# Round-4: the GPU suite on the product (cache batches of 4 for N >= 5), then the 10v10 A/B of
# 4 LDS record slots (variant "k10", -DFUTBOL_K10=4: 39.9 KB per block, still 4 blocks per CU)
# against 2 (product), with the instance matrix and v1 parity on the variant.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_k10_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_k10_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
step suite_prod 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread
FUTBOL_LIB_VARIANT=k10 step suite_k10 600 python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread
step p_10v10 200 $B --players 10 --steps 600
FUTBOL_LIB_VARIANT=k10 step k_10v10 200 $B --players 10 --steps 600
step p_10v10_b 200 $B --players 10 --steps 600
FUTBOL_LIB_VARIANT=k10 step k_10v10_b 200 $B --players 10 --steps 600
step p_2v2 200 $B
step p_5v5 200 $B --players 5 --steps 1200
