# bench A/B of two library builds: bash tools/gpu_ab_lib.sh LIB_A LIB_B [runs]
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
A=$1; B=$2; RUNS=${3:-2}
for r in $(seq $RUNS); do for L in $A $B; do
  SVO_GPU_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); p=d['phase_ms_per_step']; print('$L', d['value'], d['ms_per_step'], 'lk', p['lk'], 'fast', p['fast'], 'pyr', p['pyramid'])"
done; done
