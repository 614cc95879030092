#!/bin/bash
# Round-4 GPU diagnostics: the instance matrix (N >= 6) on the product build and on diagnostic variants,
# then the envs_v1 parity suite and the benches.  A step that fails its tests goes on to the next; a GPU
# fault (HIP error / illegal address / abort / timeout) ends the script there.
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_diag_steps.txt
    if [ $rc -ge 2 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_diag_steps.txt
        exit 1
    fi
}
PYT="python -u -m pytest -q --timeout 250 --timeout-method thread"
step inst_product 300 $PYT "tests/test_gpu_instances.py" -k "6 or 7 or 8 or 9 or 10"
FUTBOL_LIB_VARIANT=pg step inst_powglobal 300 $PYT "tests/test_gpu_instances.py" -k "6"
FUTBOL_LIB_VARIANT=ilp6 step inst_ilp6 300 $PYT "tests/test_gpu_instances.py" -k "6"
step v1_parity 400 $PYT tests/test_gpu_v1_parity.py tests/test_gpu_api.py tests/test_gpu_fullsize.py
step bench_2v2 300 python bench.py --no-rollout-line
step bench_5v5 200 python bench.py --players 5 --steps 1200 --no-cpu-baseline --no-rollout-line
step bench_10v10 200 python bench.py --players 10 --steps 600 --no-cpu-baseline --no-rollout-line
FUTBOL_SHARE_DEVICE=1 FUTBOL_DIST_BACKEND=gloo step bench_2rank 200 python bench.py --gpus 2 --steps 300 --no-cpu-baseline --no-rollout-line
