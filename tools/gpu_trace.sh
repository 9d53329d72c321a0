cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for g in 1 2; do timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tr_g$g -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --seq 64 --no-cpu-baseline --no-single --groups $g > gpurun_out/tr_g$g.log 2>&1 || exit 1; done
ls gpurun_out/tr_g1
