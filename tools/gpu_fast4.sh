# FAST v4: parity of every form, frontend parity with v4, instruction counts, bench A/B
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fast" > gpurun_out/fast4_tests.log 2>&1 || { tail -30 gpurun_out/fast4_tests.log; exit 1; }
tail -1 gpurun_out/fast4_tests.log
SVO_FAST_V=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_frontend_gpu.py tests/test_tracking_gpu.py > gpurun_out/fast4_fe.log 2>&1 || { tail -30 gpurun_out/fast4_fe.log; exit 1; }
tail -1 gpurun_out/fast4_fe.log
bash tools/gpu_pmc_env.sh "fast_detect" "SVO_FAST_V=2" "SVO_FAST_V=4" || exit 1
bash tools/gpu_ab_env_args.sh 3 "SVO_FAST_V=2|" "SVO_FAST_V=4|"
