# diagnostic: the 5v5 instance built with phi-node-folding threshold 20 (libfutbol_amd_phi5.so,
# FUTBOL_BUILD_VARIANT=phi5 FUTBOL_PHI_EXTRA=futbol_v1_n5_e64.hip) through the 5v5 GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/phi5
mkdir -p $O
FUTBOL_LIB_VARIANT=phi5 timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_v1_parity.py -v \
    -k "5v5 or 5-" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_phi5.log 2>&1
echo "phi5 rc=$?"
FUTBOL_LIB_VARIANT=phi5 timeout -k 10 300 python scripts/phi5_diag.py > $O/diag.log 2>&1
echo "diag rc=$?"
