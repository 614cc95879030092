#!/bin/bash
# Round-4 GPU check of the product build: the GPU suite, then the C2 / C5 / 10v10 bench lines.  A GPU
# fault ends the script (see gpu_r04_diag.sh).
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_check_steps.txt
    if [ $rc -ge 2 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_check_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
step ck_suite 500 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread
step ck_2v2 200 $B
step ck_5v5 200 $B --players 5 --steps 1200
step ck_10v10 200 $B --players 10 --steps 600
step ck_10v10_32k 200 $B --players 10 --steps 600 --envs 32768
