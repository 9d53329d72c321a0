# LK variant timing: bash tools/gpu_lkvar.sh TESTSEL "ENV1=a ENV2=b" "ENV1=c" ...  (parity first)
# TESTSEL: pytest -k expression over tests/ -m gpu ("all" = the whole GPU suite)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out
SEL=$1; shift
if [ "$SEL" = "all" ]; then K=""; else K="-k $SEL"; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x $K --timeout 120 --timeout-method thread -p no:cacheprovider > $O/lkvar_tests.log 2>&1 || { tail -30 $O/lkvar_tests.log; exit 1; }
tail -1 $O/lkvar_tests.log
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/lkvar$i -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 5 > $O/lkvar$i.log 2>&1 || { tail -20 $O/lkvar$i.log; exit 1; }
  python -c "
import csv,glob
for f in glob.glob('$O/lkvar$i/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_' in r['Name'] or 'pad' in r['Name']: print('$v', r['Name'][30:75], r['Calls'], r['AverageNs'], r['MinNs'])"
done
