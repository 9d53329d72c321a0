# Standalone LK kernel time (128k features, microbench) under rocprofv3 for each
# library build given (run from the repo root on the box):
#   bash tools/lk_ab.sh LIB1 LIB2 ...   (repeated alternately REPS times, default 2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in $(seq ${REPS:-2}); do for lib in "$@"; do
    T=/tmp/lkab_$(basename $lib .so)_$r
    SVO_GPU_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $T -o run --output-format csv -- \
        python tools/microbench.py lk --points 128000 --reps 6 > $T.log 2>&1 || { tail -20 $T.log; exit 1; }
    python3 - $T $(basename $lib) <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'lk_multi' in r['Name']:
        print(sys.argv[2], r['Calls'], 'avg_us', round(float(r['AverageNs']) / 1e3, 1), 'min_us', round(float(r['MinNs']) / 1e3, 1))
P
done; done
