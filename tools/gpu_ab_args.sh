# bench A/B over bench.py argument sets: bash tools/gpu_ab_args.sh "args1" "args2" [runs]
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
A1=$1; A2=$2; RUNS=${3:-2}
for r in $(seq $RUNS); do for a in "$A1" "$A2"; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single $a > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); p=d['phase_ms_per_step']; print('[$a]', d['value'], d['ms_per_step'], 'lk', p['lk'])"
done; done
