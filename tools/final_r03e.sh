set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu.sh prof r03e -- pmc r03e kitti 128 -- mix r03e || exit 1
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_r03e.log 2>&1 || { tail -20 gpurun_out/bench_r03e.log; exit 1; }
tail -1 gpurun_out/bench_r03e.log | cut -c1-400
for c in 1080p 4k; do
  timeout -k 10 400 python bench.py --config $c --seq 16 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r03e_$c.log 2>&1 || { tail -20 gpurun_out/bench_r03e_$c.log; exit 1; }
  tail -1 gpurun_out/bench_r03e_$c.log | cut -c1-300
done
