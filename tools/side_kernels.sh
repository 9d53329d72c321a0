# Standalone kernel breakdown + instruction mix of the batched pyramid chain and
# FAST detection (256 sequences, KITTI size): bash tools/side_kernels.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
tag=${1:-x}
for w in fepyr fefast; do
    rm -rf /tmp/sk_$w
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/sk_$w -o run --output-format csv -- \
        python tools/microbench.py $w --seq 256 --reps 20 > $O/sk_$w.log 2>&1 || { echo FAIL $w; tail -20 $O/sk_$w.log; exit 1; }
    tail -2 $O/sk_$w.log
    f=$(find /tmp/sk_$w -name "run_kernel_stats.csv" | head -1)
    cp $f $O/side_${tag}_${w}_kernel_stats.csv
    python - $f <<'P'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"  {r['Name'][:72]:72s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:8.2f}")
P
done
bash tools/gpu.sh mix side_$tag --cmd python tools/microbench.py fepyr --seq 256 --reps 20 | grep -E 'pyr_'
bash tools/gpu.sh mix side_$tag --cmd python tools/microbench.py fefast --seq 256 --reps 20 | grep -E 'fast_'
