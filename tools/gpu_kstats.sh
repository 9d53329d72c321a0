# Per-kernel stats per env variant: bash tools/gpu_kstats.sh PATTERN "ENV" "ENV" ...
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PAT=$1; shift; i=0
for v in "$@"; do i=$((i+1)); T=/tmp/ks_$i
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single > $T.log 2>&1 || { tail -5 $T.log; exit 1; }
  S=$(find $T -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "$PAT" $S | cut -c1-220 || true
done
