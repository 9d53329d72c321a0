# LK waves per CU vs the kernels beside it (LDS carve pad) and the sequences-per-GPU curve -- run from the repo root on the box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu.sh ab SVO_LK_LDS_PAD "0 512 1024 3072" 2 || exit 1
for s in 384 512; do
    timeout -k 10 300 python bench.py --seq $s --steps 20 --warmup 5 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order --no-forward --no-orb --no-stream > gpurun_out/seq.log 2>&1 || { tail -20 gpurun_out/seq.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/seq.log').read().strip().splitlines()[-1]); print('seq $s', d['value'], d['ms_per_step'], 'lk', d['roofline']['avg_launch_us'])"
done
