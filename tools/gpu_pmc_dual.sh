cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
MB="python tools/microbench.py lk --points 128000 --reps 2"
for q in 0 1; do
SVO_LK_QUAD=$q timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/dpmc1_$q -o run --output-format csv -- $MB > gpurun_out/dpmc.log 2>&1 &&
SVO_LK_QUAD=$q timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/dpmc2_$q -o run --output-format csv -- $MB >> gpurun_out/dpmc.log 2>&1 || { tail -20 gpurun_out/dpmc.log; exit 1; }
done
python - <<'P'
import csv, glob, collections
for q in (0, 1):
    agg = collections.defaultdict(float)
    name = None
    for f in glob.glob(f'gpurun_out/dpmc*_{q}/**/run_counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'lk_' not in r['Kernel_Name']: continue
            name = r['Kernel_Name'][:40]
            agg[r['Counter_Name']] += float(r['Counter_Value'])
    w = agg.get('SQ_WAVES', 1)
    feats = 2 * 128000 if True else 1
    print(q, name, ' '.join(f"{c}={v/feats:.0f}" for c, v in sorted(agg.items())), f"waves={w:.0f}")
P
