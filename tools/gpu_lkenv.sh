# standalone LK kernel time (microbench 128k pts, frontend criteria) per env variant
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
i=0
for v in "$@"; do i=$((i+1)); T=/tmp/lke_$i
  env $v timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $T -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 4 > $T.log 2>&1 || { tail -5 $T.log; exit 1; }
  python - $T "$v" <<'P'
import csv, glob, sys
dur = []
for f in glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']: dur.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
print(sys.argv[2], 'lk us', [round(d, 1) for d in dur])
P
done
