cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for r in 1 2; do for th in 16 14 12 8; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single --threads $th > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); p=d['phase_ms_per_step']; s=d['stats_per_step']; print('threads $th', d['value'], d['ms_per_step'], 'lk', p['lk'], 'fast', p['fast'], 'hyp', s['host_ms_hyp'], 'wait', s['host_ms_wait'])"
done; done
