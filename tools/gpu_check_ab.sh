# parity suite, then standalone LK (prev vs new lib), bench A/B libs and the polling-wait switch
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/chk_tests.log 2>&1 || { tail -30 gpurun_out/chk_tests.log; exit 1; }
tail -1 gpurun_out/chk_tests.log
bash tools/gpu_lkenv.sh "SVO_GPU_LIB=$PWD/svo_amd/lib/libsvo_gpu_prev.so" "SVO_GPU_LIB=$PWD/svo_amd/lib/libsvo_gpu.so" || exit 1
bash tools/gpu_ab_env_args.sh 2 "SVO_GPU_LIB=$PWD/svo_amd/lib/libsvo_gpu_prev.so|" "SVO_FE_SPIN=0|" "SVO_FE_SPIN=1|"
