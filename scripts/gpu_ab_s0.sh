# A/B: LLVM's default machine scheduler (variant s0) against the head build, plus the 5v5 stamps of the head build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab3 gpurun_out/st
OUT_DIR=ab3 AB="s0:--players,5 main:--players,5 s0:--players,5 main:--players,5 s0: main: s0: main: s0:--players,3 main:--players,3" bash scripts/gpu_ab.sh && \
timeout -k 10 300 python bench.py --stamps --players 5 --warmup 150 --steps 60 --profile-steps 10 --snapshots 20 --snapshot-stride 3 > gpurun_out/st/stamps5_head.log 2>&1
echo rc=$?
