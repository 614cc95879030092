# parity suite of the default library, then an A/B (2v2 and 5v5) against the variant "head"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/abt/pytest.log 2>&1 && \
VARIANTS="head default" AB_OUT=abt2 bash scripts/gpu_ab.sh && BENCH_ARGS="--players 5" VARIANTS="head default" AB_OUT=abt5 bash scripts/gpu_ab.sh
echo rc=$?
