# bench --legs first vs after under rocprofv3 --kernel-trace (the headline's step
# timeline in both orders), restricted side legs: forward + bucketed
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
for legs in first after; do
    rm -rf $O/legs_$legs
    timeout -k 10 400 rocprofv3 --kernel-trace -d $O/legs_$legs -o run --output-format csv -- \
        python bench.py --steps 20 --warmup 5 --legs $legs --no-cpu-baseline --no-single --no-orb --no-stream \
        --no-opencv-order > $O/legs_$legs.log 2>&1 || { echo "FAILED $legs"; tail -20 $O/legs_$legs.log; exit 1; }
    tail -1 $O/legs_$legs.log | cut -c1-400
done
