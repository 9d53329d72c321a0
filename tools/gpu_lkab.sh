# A/B of the LK kernels (rocprofv3 kernel stats over the microbenchmark).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for cfg in "0 4" "1 4" "1 1"; do set -- $cfg
  rm -rf gpurun_out/lkab
  SVO_LK_QUAD=$1 SVO_LK_DUAL_MINW=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lkab -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 6 > gpurun_out/lkab.log 2>&1 || { tail -5 gpurun_out/lkab.log; exit 1; }
  python - "$1" "$2" <<'P'
import csv, glob, sys
f = glob.glob('gpurun_out/lkab/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'lk_' in r['Name']:
        print(f"dual={sys.argv[1]} minw={sys.argv[2]} {r['Name'][:50]} calls={r['Calls']} avg_us={float(r['AverageNs'])/1e3:.1f} min_us={float(r['MinNs'])/1e3:.1f}")
P
done
