# OpenCV-order LK kernel time (128k features, microbench --cv) per library build,
# alternated (run from the repo root on the box): bash tools/cv_ab.sh LIB1 LIB2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in $(seq ${REPS:-2}); do for lib in "$@"; do
    T=/tmp/cvab_$(basename $lib .so)_$r
    SVO_GPU_LIB=$PWD/$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $T -o run --output-format csv -- \
        python tools/microbench.py lk --points 128000 --reps 3 --cv > $T.log 2>&1 || { tail -20 $T.log; exit 1; }
    python3 - $T $(basename $lib) <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'lk_cv' in r['Name']:
        print(sys.argv[2], r['Name'][40:75], r['Calls'], 'avg_us', round(float(r['AverageNs']) / 1e3, 1))
P
done; done
