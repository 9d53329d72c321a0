# FAST v3 check: parity of every detection form, frontend parity with v3, bench A/B
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fast" > gpurun_out/fast3_tests.log 2>&1 || { tail -30 gpurun_out/fast3_tests.log; exit 1; }
tail -2 gpurun_out/fast3_tests.log
SVO_FAST_V=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_frontend_gpu.py tests/test_tracking_gpu.py > gpurun_out/fast3_fe.log 2>&1 || { tail -30 gpurun_out/fast3_fe.log; exit 1; }
tail -2 gpurun_out/fast3_fe.log
bash tools/gpu_ab_env_args.sh 2 "SVO_FAST_V=2|" "SVO_FAST_V=3|"
