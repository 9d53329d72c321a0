cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x --timeout 300 -p no:cacheprovider -k "lk" > gpurun_out/quad_tests.log 2>&1 || { tail -40 gpurun_out/quad_tests.log; exit 1; }
tail -2 gpurun_out/quad_tests.log
for cfg in "0 4" "1 1" "1 4"; do set -- $cfg; SVO_LK_QUAD=$1 SVO_LK_DUAL_MINW=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-single > gpurun_out/bq.log 2>&1 || { tail -5 gpurun_out/bq.log; exit 1; }; python -c "
import json; d=json.loads(open('gpurun_out/bq.log').read().strip().splitlines()[-1]); print('dual=$1 minw=$2', d['value'], d['ms_per_step'], d['phase_ms_per_step']['lk'])"; done
