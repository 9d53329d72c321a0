set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
B="python bench.py --seq 256 --steps 6 --warmup 2 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order --no-forward --no-orb"
for v in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf /tmp/pab_$c_$v
    SVO_XCD_TILES=$v timeout -s KILL 200 rocprofv3 --pmc $c -d /tmp/pab_${c}_$v -o run --output-format csv -- $B > $O/pab.log 2>&1 || { echo FAIL; tail -20 $O/pab.log; exit 1; }
    python - /tmp/pab_${c}_$v $v $c <<'P'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/run_counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(float); n = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    if 'fast_detect' in k or 'pyr_scharr' in k:
        k = k[:60]; agg[k] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k in agg: print('XCD', sys.argv[2], sys.argv[3], k, 'MB/launch', round(agg[k] * 1024 / len(n[k]) / 1e6, 1), 'launches', len(n[k]))
P
  done
done
