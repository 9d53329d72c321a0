# bench A/B over env+args sets: bash tools/gpu_ab_env_args.sh RUNS "ENV args" "ENV args" ...
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
RUNS=$1; shift
for r in $(seq $RUNS); do for v in "$@"; do
  env ${v%%|*} timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single ${v#*|} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('[$v]', d['value'], d['ms_per_step'])"
done; done
