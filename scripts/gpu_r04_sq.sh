#!/bin/bash
# Round-4: the cost of the exact squares (A/B of the product against the psq diagnostic build, whose
# squares are x*x with the same batching), and the per-phase stamps of the 2v2 / 5v5 step kernels.
mkdir -p gpurun_out/st
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_sq_steps.txt
    if [ $rc -ge 2 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_sq_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
step sq_prod_a 200 $B
FUTBOL_LIB_VARIANT=psq step sq_psq_a 200 $B
step sq_prod_b 200 $B
FUTBOL_LIB_VARIANT=psq step sq_psq_b 200 $B
step sq_prod_5 200 $B --players 5 --steps 1200
FUTBOL_LIB_VARIANT=psq step sq_psq_5 200 $B --players 5 --steps 1200
step st_2v2 300 python bench.py --stamps --warmup 150 --steps 100 --profile-steps 10 --snapshots 60 --snapshot-stride 3 --stamps-dump gpurun_out/st/waves2.npy
step st_5v5 300 python bench.py --stamps --players 5 --warmup 150 --steps 60 --profile-steps 10 --snapshots 40 --snapshot-stride 3 --stamps-dump gpurun_out/st/waves5.npy
