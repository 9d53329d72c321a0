# bench A/B of an env toggle: bash tools/gpu_ab.sh VAR "v1 v2" [runs]
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2; RUNS=${3:-2}
for r in $(seq $RUNS); do for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); p=d['phase_ms_per_step']; print('$VAR=$v', d['value'], d['ms_per_step'], 'lk', p['lk'], 'fast', p['fast'], 'pyr', p['pyramid'])"
done; done
