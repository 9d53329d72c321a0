cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x --timeout 300 -p no:cacheprovider -k "lk" > gpurun_out/lk_tests.log 2>&1 || { tail -30 gpurun_out/lk_tests.log; exit 1; }
tail -2 gpurun_out/lk_tests.log
for m in 1; do SVO_LK_MINW=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m$m -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 4 > gpurun_out/mb$m.log 2>&1 || exit 1; done
for m in 1; do echo "minw $m $(grep lk_fast gpurun_out/prof_m$m/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f3)"; done
