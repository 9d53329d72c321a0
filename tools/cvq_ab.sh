# OpenCV-order LK (128k features, microbench --cv, 21x21) four per wave (lk_cvq_kernel)
# vs one per wave (SVO_LK_QUAD=0: lk_cv_kernel), alternated, under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# (LIBS: library builds to alternate, default the in-tree one)
for r in $(seq ${REPS:-2}); do for lib in ${LIBS:-svo_amd/lib/libsvo_gpu.so}; do for q in ${QUADS:-1 0}; do
    T=/tmp/cvq_${q}_$(basename $lib .so)_$r
    SVO_GPU_LIB=$PWD/$lib SVO_LK_QUAD=$q timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $T -o run --output-format csv -- \
        python tools/microbench.py lk --points 128000 --reps 3 --cv > $T.log 2>&1 || { tail -20 $T.log; exit 1; }
    python3 - $T $q $(basename $lib) <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'lk_cv' in r['Name']:
        print(sys.argv[3], 'SVO_LK_QUAD=' + sys.argv[2], r['Name'][40:80], r['Calls'], 'avg_us', round(float(r['AverageNs']) / 1e3, 1))
P
done; done; done
