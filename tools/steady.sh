# Steady-state check of the driver's exact bench window (--steps 20 --warmup 5):
# RUNS runs of bench.py's headline leg, each line's step times and slowest step.
#   bash tools/steady.sh [RUNS] [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
runs=${1:-3}; shift
for r in $(seq $runs); do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order --no-forward --no-orb "$@" \
        > $O/steady_$r.log 2>&1 || { echo "FAILED run $r"; tail -30 $O/steady_$r.log; exit 1; }
    python - $O/steady_$r.log <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sm = d["step_ms"]
print("value", d["value"], "ms/step", d["ms_per_step"], "mean", sm["mean"], "median", sm["median"], "max", sm["max"])
print("  steps", sm["all"])
print("  slowest", json.dumps(d["slowest_step"]))
print("  per step", json.dumps(d["stats_per_step"]))
P
done
