cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
grep -m1 "model name" /proc/cpuinfo; grep -o -m1 "avx2" /proc/cpuinfo; nproc
timeout -k 10 600 python -m pytest tests/test_frontend_gpu.py tests/test_gpu_parity.py tests/test_tracking_gpu.py -q -x --timeout 300 -p no:cacheprovider > gpurun_out/fe_tests.log 2>&1 || { tail -30 gpurun_out/fe_tests.log; exit 1; }
tail -2 gpurun_out/fe_tests.log
rm -f gpurun_out/bench_g.log
for g in 1; do timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-single --groups $g >> gpurun_out/bench_g.log 2>&1 || exit 1; done
python - <<'P'
import json
for l in open('gpurun_out/bench_g.log'):
    if l.startswith('{'):
        d=json.loads(l); st=d['stats_per_step']; print(d['config'].get('groups'), d['value'], d['ms_per_step'], d['phase_ms_per_step']['lk'], st['host_ms_hyp'], st['host_ms_fit'], st['host_ms_wait'], d['roofline']['avg_launch_us'])
P
