# Headline frames/s vs sequences per GPU (the driver's window: --steps 20 --warmup 5)
#   bash tools/seqcurve.sh "128 192 256" [RUNS]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
for r in $(seq ${2:-1}); do for s in $1; do
    timeout -k 10 400 python bench.py --seq $s --steps 20 --warmup 5 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order \
        --no-forward --no-orb > $O/seq_$s.log 2>&1 || { echo "FAILED seq $s"; tail -20 $O/seq_$s.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/seq_$s.log').read().strip().splitlines()[-1]); sm=d['step_ms']
print('seq', $s, d['value'], 'ms/step', d['ms_per_step'], 'median', sm['median'], 'max', sm['max'], 'lk_us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'])"
done; done
