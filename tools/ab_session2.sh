# LK tail A/B (duo + single tails, 4 vs 3 waves per SIMD) -- run from the repo root on the box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/svo_amd/lib
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_frontend_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/ab2_tests.log 2>&1 || { tail -30 $O/ab2_tests.log; exit 1; }
tail -1 $O/ab2_tests.log
LKAB_VAR=SVO_GPU_LIB bash tools/gpu.sh lkab "$L/libsvo_gpu_single.so $L/libsvo_gpu.so $L/libsvo_gpu_m3.so" || exit 1
LKAB_VAR=SVO_LK_TAIL bash tools/gpu.sh lkab "1 2" || exit 1
AB_STEPS=30 bash tools/lib_ab.sh 1 svo_amd/lib/libsvo_gpu_single.so svo_amd/lib/libsvo_gpu.so svo_amd/lib/libsvo_gpu_m3.so || exit 1
AB_STEPS=30 AB_ARGS="--scene forward" bash tools/lib_ab.sh 1 svo_amd/lib/libsvo_gpu_single.so svo_amd/lib/libsvo_gpu.so svo_amd/lib/libsvo_gpu_m3.so || exit 1
