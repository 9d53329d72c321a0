# SQ counters of the FAST / pyramid kernels over a short bench run (separate --pmc passes).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
B="python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-single"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/fpmc1 -o run --output-format csv -- $B > gpurun_out/fpmc.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH -d gpurun_out/fpmc2 -o run --output-format csv -- $B >> gpurun_out/fpmc.log 2>&1 || { tail -20 gpurun_out/fpmc.log; exit 1; }
python - <<'P'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(int)
for f in glob.glob('gpurun_out/fpmc*/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:50]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    if not any(s in k for s in ('fast_', 'pyr_', 'box_bin', 'scharr', 'lk_fast')): continue
    w = d.get('SQ_WAVES', 1) or 1
    print(k)
    print('   ' + ' '.join(f"{c}={v/w:.1f}" for c, v in sorted(d.items()) if c != 'SQ_WAVES') + f" waves={w:.0f}")
P
