# Kernel-time profile of a short bench run (rocprofv3 kernel trace + stats).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out
rm -rf $O/prof_quick
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_quick -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-single > $O/prof_quick.log 2>&1 || { tail -20 $O/prof_quick.log; exit 1; }
python - <<'P'
import csv, glob
f = glob.glob('gpurun_out/prof_quick/**/run_kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:25]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.2f} total_ms={float(r['TotalDurationNs'])/1e6:8.2f} pct={r['Percentage']}")
P
