# LK VALU split: setup (iteration cap 1) vs full, standalone microbench
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for c in 1 2 50; do T=/tmp/lks_$c
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM -d $T -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 2 --count $c > $T.log 2>&1 || { tail -5 $T.log; exit 1; }
  timeout -k 10 90 rocprofv3 --kernel-trace --stats -d ${T}k -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 3 --count $c >> $T.log 2>&1 || { tail -5 $T.log; exit 1; }
  python - $T $c <<'P'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + '/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']: agg[r['Counter_Name']] += float(r['Counter_Value'])
dur = []
for f in glob.glob(sys.argv[1] + 'k/**/run_kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']: dur.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
print('count', sys.argv[2], 'us', [round(d, 1) for d in dur], ' '.join(f"{k}={v/2/128000*4:.0f}/wave" for k, v in sorted(agg.items())))
P
grep iters $T.log | tail -1
done
