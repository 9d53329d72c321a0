# final-build checks: smoke, the N=2 multi-rank path on the one-GPU box (ranks share GPU 0) -- run from the repo root on the box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu.sh smoke || exit 1
timeout -k 10 400 python bench.py --gpus 2 --seq 128 --steps 10 --warmup 3 --no-cpu-baseline --no-single --no-bucketed \
    --no-opencv-order --no-forward --no-orb --no-stream > gpurun_out/n2.log 2>&1 || { tail -30 gpurun_out/n2.log; exit 1; }
tail -1 gpurun_out/n2.log | cut -c1-700
