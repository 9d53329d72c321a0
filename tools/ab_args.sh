# Alternated bench A/B of two argument sets (run from the repo root on the box):
#   bash tools/ab_args.sh RUNS "ARGS_A" "ARGS_B"
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
runs=$1; shift
for r in $(seq $runs); do for a in "$@"; do
    timeout -k 10 200 python bench.py --steps ${AB_STEPS:-40} --warmup 5 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order \
        --no-forward --no-orb $a > gpurun_out/ab_args.log 2>&1 || { tail -20 gpurun_out/ab_args.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab_args.log').read().strip().splitlines()[-1]); sm=d.get('step_ms', {})
print('[$a]', d['value'], d['ms_per_step'], 'median', sm.get('median'), 'p90', sm.get('p90'), 'lk_us', d['roofline']['avg_launch_us'])"
done; done
