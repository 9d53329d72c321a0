cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_frontend_gpu.py -q --timeout 300 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; echo EXIT $? >> gpurun_out/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lk -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 5 > gpurun_out/prof_lk.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM -d gpurun_out/pmc_lk -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 2 >> gpurun_out/prof_lk.log 2>&1
for S in 1 64; do timeout -k 10 300 python bench.py --steps 10 --warmup 2 --seq $S --no-cpu-baseline --no-single >> gpurun_out/bench.log 2>&1; done
