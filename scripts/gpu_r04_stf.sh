#!/bin/bash
# Round-4 stamps of the final step kernels (diagnostic build FUTBOL_BUILD_VARIANT=stamps): 10v10, 5v5, 2v2.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_stf_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_stf_steps.txt
        exit 1
    fi
}
step stf_10v10 300 python bench.py --stamps --players 10 --warmup 150 --steps 30 --profile-steps 5 --snapshots 20 --snapshot-stride 3
step stf_5v5 300 python bench.py --stamps --players 5 --warmup 150 --steps 60 --profile-steps 10 --snapshots 40 --snapshot-stride 3
step stf_2v2 300 python bench.py --stamps --warmup 150 --steps 100 --profile-steps 10 --snapshots 60 --snapshot-stride 3
