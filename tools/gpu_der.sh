# pair-record derivative layout: parity (LK / pyramid / frontend) then A/B vs the previous build
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/der_tests.log 2>&1 || { tail -30 gpurun_out/der_tests.log; exit 1; }
tail -2 gpurun_out/der_tests.log
bash tools/gpu_ab_lib.sh svo_amd/lib/libsvo_gpu_prev.so svo_amd/lib/libsvo_gpu.so 2
