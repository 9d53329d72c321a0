# bench --legs first vs after (restricted side legs: forward + bucketed); with
# PROF=1 each under rocprofv3 --kernel-trace (the headline's step timeline in both
# orders: python tools/step_timeline.py gpurun_out/legs_first --first -6)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
for legs in ${LEGS:-first after}; do
    pre=""
    if [ "${PROF:-0}" = 1 ]; then
        rm -rf $O/legs_$legs
        pre="rocprofv3 --kernel-trace -d $O/legs_$legs -o run --output-format csv --"
    fi
    timeout -k 10 400 $pre python bench.py --steps 20 --warmup 5 --legs $legs --no-cpu-baseline --no-single \
        --no-orb --no-stream --no-opencv-order > $O/legs_$legs.log 2>&1 || { echo "FAILED $legs"; tail -20 $O/legs_$legs.log; exit 1; }
    python3 -c "
import json
d = json.loads([x for x in open('$O/legs_$legs.log').read().splitlines() if x.startswith('{')][-1])
sl = d['slowest_step']
print('legs $legs', d['value'], d['ms_per_step'], 'bucketed', (d['bucketed'] or {}).get('value'), 'forward',
      d['workloads']['forward']['value'], 'slowest: fit', sl['host_ms_fit'], 'wait_post', sl['host_ms_wait_post'])"
done
