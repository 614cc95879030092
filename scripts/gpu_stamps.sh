set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --stamps --warmup 100 --steps 190 --profile-steps 10 > gpurun_out/stamps.log 2>&1
