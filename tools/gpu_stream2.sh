# full GPU suite (default), frontend parity with the streamed mode, then A/B
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
SVO_FE_STREAM=1 SVO_FE_FAST_PRIO=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_frontend_gpu.py tests/test_tracking_gpu.py > gpurun_out/stream_fe.log 2>&1 || { tail -30 gpurun_out/stream_fe.log; exit 1; }
tail -1 gpurun_out/stream_fe.log
bash tools/gpu_ab_env_args.sh 3 "SVO_FE_STREAM=0|" "SVO_FE_STREAM=1|" "SVO_FE_STREAM=1 SVO_FE_FAST_PRIO=1|"
