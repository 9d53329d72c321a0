cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tr_g1 -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --seq 64 --no-cpu-baseline --no-single > gpurun_out/tr_g1.log 2>&1 || exit 1
