# PMC instruction mix of every kernel of the batched step (bench.py), per dispatch.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out
B="python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-single"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM -d /tmp/ps1 -o run --output-format csv -- $B > $O/ps.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d /tmp/ps2 -o run --output-format csv -- $B >> $O/ps.log 2>&1 || { tail -20 $O/ps.log; exit 1; }
python - <<'P'
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob('/tmp/ps[12]/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r'([a-z_0-9]+_kernel)', r['Kernel_Name'])
        if not m: continue
        k = m.group(1)
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add((f, r['Dispatch_Id']))
for k, d in agg.items():
    n = len(disp[k]) / 2
    w = d.get('SQ_WAVES', 1)
    print(f"{k:28s} disp {n:5.0f} waves/disp {w/n:9.0f} | per wave: " + ' '.join(f"{c.replace('SQ_','')}={v/w:.0f}" for c, v in sorted(d.items()) if c != 'SQ_WAVES'))
P
