set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/svo_amd/lib
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_frontend_gpu.py tests/test_tracking_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/ab1_tests.log 2>&1 || { tail -30 $O/ab1_tests.log; exit 1; }
tail -1 $O/ab1_tests.log
LKAB_VAR=SVO_GPU_LIB bash tools/gpu.sh lkab "$L/libsvo_gpu_head.so $L/libsvo_gpu.so" || exit 1
LKAB_VAR=SVO_LK_TAIL bash tools/gpu.sh lkab "0 1" || exit 1
bash tools/lib_ab.sh 2 svo_amd/lib/libsvo_gpu_head.so svo_amd/lib/libsvo_gpu.so || exit 1
AB_ARGS="--scene forward" bash tools/lib_ab.sh 2 svo_amd/lib/libsvo_gpu_head.so svo_amd/lib/libsvo_gpu.so || exit 1
