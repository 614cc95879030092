# stamps tail study for 5v5 and 2v2 (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/st
timeout -k 10 300 python bench.py --stamps --players 5 --warmup 150 --steps 60 --profile-steps 10 --snapshots 40 --snapshot-stride 3 --stamps-dump gpurun_out/st/waves5.npy > gpurun_out/st/stamps5.log 2>&1 && \
timeout -k 10 300 python bench.py --stamps --warmup 150 --steps 100 --profile-steps 10 --snapshots 60 --snapshot-stride 3 --stamps-dump gpurun_out/st/waves2.npy > gpurun_out/st/stamps2.log 2>&1
echo rc=$?
