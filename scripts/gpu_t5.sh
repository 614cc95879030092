set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t5
for v in default nophi; do vv=$v; [ "$v" = default ] && vv=""; FUTBOL_LIB_VARIANT=$vv timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -k "episode_lengths" tests/test_gpu_v1_parity.py -k "episode_lengths or free_running" -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t5/$v.log 2>&1; echo "$v rc=$?"; done
