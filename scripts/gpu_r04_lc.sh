#!/bin/bash
# Round-4 A/B: the preloaded arbiter-cache entries loaded after the action phase too (variant
# "latec", every N) against the product (late v_bias for N >= 5); full GPU suite on the product,
# instance matrix + v1 parity on the variant.
mkdir -p gpurun_out
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/r04_lc_steps.txt
    if [ $rc -ne 0 ] || grep -q -E "HIP error|hipError|illegal memory|Aborted|core dumped" "gpurun_out/$name.log"; then
        echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/r04_lc_steps.txt
        exit 1
    fi
}
B="python bench.py --no-cpu-baseline --no-rollout-line"
T="python -u -m pytest tests/test_gpu_instances.py tests/test_gpu_v1_parity.py -x -q --timeout 250 --timeout-method thread"
step suite_prod 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread
FUTBOL_LIB_VARIANT=latec step suite_latec 400 $T
for r in a b c; do
    step p2_$r 200 $B
    FUTBOL_LIB_VARIANT=latec step c2_$r 200 $B
    step p5_$r 200 $B --players 5 --steps 1200
    FUTBOL_LIB_VARIANT=latec step c5_$r 200 $B --players 5 --steps 1200
done
step p10_a 200 $B --players 10 --steps 600
FUTBOL_LIB_VARIANT=latec step c10_a 200 $B --players 10 --steps 600
