# GPU suite, then A/B bench lines of the head build against the "base" variant (HEAD source)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${OUT_DIR:-ab1}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${OUT_DIR:-ab1}/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/${OUT_DIR:-ab1}/pytest.log; exit 1; }
tail -2 gpurun_out/${OUT_DIR:-ab1}/pytest.log
AB="${AB:-base:--players,5 main:--players,5 base:--players,5 main:--players,5 base:--players,3 main:--players,3 base:--players,10,--steps,600 main:--players,10,--steps,600 base: main:}" bash scripts/gpu_ab.sh
