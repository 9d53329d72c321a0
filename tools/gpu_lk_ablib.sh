# standalone LK kernel (microbench, 128k points) per library: duration + VALU/LDS/VMEM instruction counts
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; i=0
for L in "$@"; do i=$((i+1)); T=/tmp/lkab_$i
  SVO_GPU_LIB=$PWD/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $T -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 3 > $T.log 2>&1 || { tail -5 $T.log; exit 1; }
  SVO_GPU_LIB=$PWD/$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d ${T}p -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 2 >> $T.log 2>&1 || { tail -5 $T.log; exit 1; }
  echo "== $L"; grep -h "lk_multi" $(find $T -name "*kernel_stats.csv") | cut -d, -f1-4 | cut -c1-160
  python - ${T}p <<'P'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + '/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']: agg[r['Counter_Name']] += float(r['Counter_Value'])
print(' '.join(f"{k}={v/2/128000:.1f}/pt" for k, v in sorted(agg.items())))
P
done
