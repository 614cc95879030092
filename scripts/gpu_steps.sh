#!/bin/bash
# One GPU call = a list of steps (run through gpurun from the repo root):
#   gpurun --timeout 1200 -- bash scripts/gpu_steps.sh <steps-file> <out-dir> [section]
# Each non-empty, non-# line of <steps-file> is "NAME TIMEOUT_S COMMAND...", e.g.
#   suite   600  python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread
#   b_kx6   200  env FUTBOL_LIB_VARIANT=kx6 python bench.py --no-cpu-baseline --players 5
# A line "[name]" starts a section: with a [section] argument only that section's steps run (a round's
# calls live in one file, scripts/steps/rNN.txt, one section per call); without one, every step runs.
# Output of step NAME goes to <out-dir>/NAME.log; <out-dir>/steps.txt lists every step's status.
# A step that fails with rc 1 (a test or assertion failure) does not stop the list; a time limit
# (124 / 137), an abort (134), a segfault (139) or a HIP fault in the log ends it -- nothing more runs
# on the GPU after a fault.  (Replaces round 4's one-off scripts/gpu_r04_*.sh A/B drivers.)
# Steps read /dev/null, not the steps file (a step reading stdin would eat the remaining lines), and
# a last line without a trailing newline still runs.
set -u
steps=$1
out=${2:-gpurun_out/steps}
want=${3:-}
sec=""
mkdir -p "$out"
: > "$out/steps.txt"
while read -r name to cmd || [ -n "${name:-}" ]; do
    [ -z "${name:-}" ] && continue
    case "$name" in \#*) continue ;; esac
    case "$name" in \[*\]) sec=${name#[}; sec=${sec%]}; continue ;; esac
    if [ -n "$want" ] && [ "$sec" != "$want" ]; then continue; fi
    start=$(date +%s)
    timeout -k 10 "$to" bash -c "$cmd" > "$out/$name.log" 2>&1 < /dev/null
    rc=$?
    echo "$name rc=$rc $(( $(date +%s) - start ))s" | tee -a "$out/steps.txt"
    if grep -q -E "HIP error|hipError|illegal memory|Memory access fault|Aborted|core dumped" "$out/$name.log"; then
        echo "stopping after $name: GPU fault in the log" | tee -a "$out/steps.txt"
        exit 2
    fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)" | tee -a "$out/steps.txt"
        exit 2
    fi
done < "$steps"
exit 0
