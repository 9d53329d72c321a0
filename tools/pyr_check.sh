# Pyramid parity tests + the front end's pyramid chain timed alone (fused vs
# per-level launches) + per-kernel (name, grid) durations of both (run on the GPU box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pyramid or scharr" -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $O/pyr_tests.log 2>&1 || { tail -30 $O/pyr_tests.log; exit 1; }
tail -1 $O/pyr_tests.log
for wh in "1241 376" "1920 1080"; do set -- $wh; for f in 0 1; do
    SVO_PYR_FUSED=$f timeout -k 10 120 python tools/microbench.py fepyr --w $1 --h $2 --seq 64 --reps 50 || exit 1
done; done
for f in 0 1; do
    rm -rf $O/prof_pyr$f
    SVO_PYR_FUSED=$f timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_pyr$f -o run --output-format csv -- \
        python tools/microbench.py fepyr --w ${PYR_W:-1241} --h ${PYR_H:-376} --seq 64 --reps 50 > $O/prof_pyr$f.log 2>&1 || exit 1
    echo "SVO_PYR_FUSED=$f"
    python - $O/prof_pyr$f <<'P'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = (r['Kernel_Name'][:48], r.get('Grid_Size_X', r.get('Grid_Size', '')), r.get('Grid_Size_Y', ''))
    d[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if len(v) >= 10:
        v.sort()
        print(f"  {k[0]:48s} grid {k[1]:>6s}x{k[2]:<5s} n={len(v):4d} median_us={v[len(v)//2]:8.2f}")
P
done
