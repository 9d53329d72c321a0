# OpenCV-order LK (lk_cvq_kernel) with G + int16 d in LDS: parity, then the kernel alone and the bench leg against the
# previous layout -- run from the repo root on the box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/svo_amd/lib
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lk_opencv_order_gpu.py tests/test_tracking_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/ab7_tests.log 2>&1 || { tail -30 $O/ab7_tests.log; exit 1; }
tail -1 $O/ab7_tests.log
for lib in libsvo_gpu_cvold.so libsvo_gpu.so; do
    T=/tmp/cvq_$lib
    SVO_GPU_LIB=$L/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T -o run --output-format csv -- \
        python tools/microbench.py lk --cv --points 128000 --reps 3 > $T.log 2>&1 || { tail -20 $T.log; exit 1; }
    python3 - $T $lib <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'lk_cvq' in r['Name'] or 'lk_cv_' in r['Name']:
        print(sys.argv[2], r['Name'][40:90], r['Calls'], 'avg_us', round(float(r['AverageNs']) / 1e3, 1))
P
done
for lib in libsvo_gpu_cvold.so libsvo_gpu.so; do
    SVO_GPU_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-single --no-bucketed \
        --no-forward --no-orb --no-stream > $O/cv.log 2>&1 || { tail -20 $O/cv.log; exit 1; }
    python -c "
import json; d=json.loads(open('$O/cv.log').read().strip().splitlines()[-1]); print('$lib', 'headline', d['value'], 'opencv_order', d['workloads']['opencv_order']['value'], d['workloads']['opencv_order']['ms_per_step'])"
done
