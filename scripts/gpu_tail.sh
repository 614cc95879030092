# tail study: per-wave cycles and event counts of single step launches (stamps build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tail
timeout -k 10 300 python bench.py --stamps --warmup 150 --steps 100 --profile-steps 10 --snapshots 60 --snapshot-stride 3 \
    --stamps-dump gpurun_out/tail/waves.npy > gpurun_out/tail/stamps.log 2>&1
echo rc=$?
