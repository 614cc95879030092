set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --stamps --warmup 40 --steps 300 --profile-steps 10 --snapshots 64 > gpurun_out/stamps.log 2>&1
