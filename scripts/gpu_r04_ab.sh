#!/bin/bash
# Round-4 GPU run: the GPU suite on the product build, then A/B benches (product vs a variant library
# named by $1) and the 10v10 occupancy check.  A GPU fault ends the script (see gpu_r04_diag.sh).
mkdir -p gpurun_out
V=${1:-pa}
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_ab_steps.txt
    if [ $rc -ge 2 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_ab_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
step suite 500 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread
step ab_prod_2v2_a 200 $B
FUTBOL_LIB_VARIANT=$V step ab_var_2v2_a 200 $B
step ab_prod_2v2_b 200 $B
FUTBOL_LIB_VARIANT=$V step ab_var_2v2_b 200 $B
step ab_prod_5v5 200 $B --players 5 --steps 1200
FUTBOL_LIB_VARIANT=$V step ab_var_5v5 200 $B --players 5 --steps 1200
step occ_10v10_32k 200 $B --players 10 --steps 600 --envs 32768
step occ_10v10_48k 200 $B --players 10 --steps 600 --envs 49152
