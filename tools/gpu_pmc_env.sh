# instruction counts per call of kernels matching PAT inside the bench, per env variant:
# bash tools/gpu_pmc_env.sh PAT "ENV" "ENV" ...
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PAT=$1; shift; i=0
for v in "$@"; do i=$((i+1)); T=/tmp/pe_$i
  env $v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVES SQ_INSTS_BRANCH -d $T -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-single > $T.log 2>&1 || { tail -5 $T.log; exit 1; }
  echo "== $v"
  python - $T "$PAT" <<'P'
import csv, glob, sys, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + '/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        if not re.search(sys.argv[2], n): continue
        k = n.split('(')[0][-40:]
        agg[k][r['Counter_Name']] += float(r['Counter_Value']); calls[k].add(r['Dispatch_Id'])
for k, d in agg.items():
    nc = len(calls[k])
    print(k, 'calls', nc, ' '.join(f"{c}={v/nc:.4g}" for c, v in sorted(d.items())))
P
done
