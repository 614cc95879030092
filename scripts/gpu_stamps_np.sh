# 5v5 stamps: the shipped source vs the no-pass-draw diagnostic (wrong results; cost of the pass-target draws)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/st
FUTBOL_LIB_VARIANT=stampsnp timeout -k 10 300 python bench.py --stamps --players 5 --warmup 150 --steps 60 --profile-steps 10 --snapshots 20 --snapshot-stride 3 > gpurun_out/st/stamps5_np.log 2>&1
echo rc=$?
