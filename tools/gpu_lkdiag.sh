# LK dual-kernel diagnosis: PMC instruction mix per feature + time vs iteration cap.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out
MB="python tools/microbench.py lk --points 128000 --reps 2"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM -d $O/lkd1 -o run --output-format csv -- $MB > $O/lkd.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d $O/lkd2 -o run --output-format csv -- $MB >> $O/lkd.log 2>&1 || { tail -20 $O/lkd.log; exit 1; }
for c in 1 2 4 50; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/lkc$c -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 3 --count $c >> $O/lkd.log 2>&1 || { tail -20 $O/lkd.log; exit 1; }
done
python - <<'P'
import csv, glob, collections
agg = collections.defaultdict(float)
for f in glob.glob('gpurun_out/lkd[12]/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_' not in r['Kernel_Name']: continue
        agg[r['Counter_Name']] += float(r['Counter_Value'])
feats = 2 * 128000
print('per feature:', ' '.join(f"{c}={v/feats:.1f}" for c, v in sorted(agg.items())))
for c in (1, 2, 4, 50):
    for f in glob.glob(f'gpurun_out/lkc{c}/**/run_kernel_stats.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'lk_' in r['Name']: print('count', c, r['Name'][:50], r['Calls'], r['AverageNs'])
P
