# New-feature GPU tests (ingest, ORB, tracking mirror) in one pytest process.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_ingest.py tests/test_orb.py tests/test_tracking_gpu.py -q -x --timeout 300 -p no:cacheprovider > gpurun_out/new_tests.log 2>&1 || { tail -40 gpurun_out/new_tests.log; exit 1; }
tail -3 gpurun_out/new_tests.log
