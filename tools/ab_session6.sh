# LK under the compiler's other scheduling strategies (lk.o only; max-memory-clause; max-ilp at 4 waves) -- run from the repo root on the box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/svo_amd/lib
LKAB_VAR=SVO_GPU_LIB bash tools/gpu.sh lkab "$L/libsvo_gpu.so $L/libsvo_gpu_mc.so $L/libsvo_gpu_ilp4.so" || exit 1
AB_STEPS=30 bash tools/lib_ab.sh 1 svo_amd/lib/libsvo_gpu.so svo_amd/lib/libsvo_gpu_mc.so svo_amd/lib/libsvo_gpu_ilp4.so || exit 1
