# Alternated bench A/B of library builds (run from the repo root on the box):
#   bash tools/lib_ab.sh RUNS LIB_A LIB_B ...   (each via SVO_GPU_LIB; headline only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
runs=$1; shift
for r in $(seq $runs); do for lib in "$@"; do
    SVO_GPU_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps ${AB_STEPS:-40} --warmup 5 --no-cpu-baseline \
        --no-single --no-bucketed --no-opencv-order --no-forward --no-orb --no-stream ${AB_ARGS:-} \
        > gpurun_out/lib_ab.log 2>&1 || { tail -20 gpurun_out/lib_ab.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/lib_ab.log').read().strip().splitlines()[-1]); sm=d.get('step_ms', {})
print('[$lib]', d['value'], d['ms_per_step'], 'median', sm.get('median'), 'p90', sm.get('p90'), 'lk_us', d['roofline']['avg_launch_us'])"
done; done
