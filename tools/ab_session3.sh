# LK setup-group / launch-bound variants at 4 waves per SIMD -- run from the repo root on the box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/svo_amd/lib
LKAB_VAR=SVO_GPU_LIB bash tools/gpu.sh lkab "$L/libsvo_gpu.so $L/libsvo_gpu_k1.so $L/libsvo_gpu_k4.so $L/libsvo_gpu_m4.so" || exit 1
AB_STEPS=30 bash tools/lib_ab.sh 1 svo_amd/lib/libsvo_gpu.so svo_amd/lib/libsvo_gpu_k4.so svo_amd/lib/libsvo_gpu_m4.so svo_amd/lib/libsvo_gpu_k1.so || exit 1
