cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
SVO_FE_TRACE=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --seq 64 --no-cpu-baseline --no-single > gpurun_out/fetrace.log 2>&1 || exit 1
grep "t=8\]" gpurun_out/fetrace.log; tail -1 gpurun_out/fetrace.log | cut -c1-200
