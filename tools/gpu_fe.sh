# Frontend + new parity tests, then a short bench (usage: bash tools/gpu_fe.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_frontend_gpu.py tests/test_ingest.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > $O/fe_tests.log 2>&1 || { echo "fe tests failed"; tail -40 $O/fe_tests.log; exit 1; }
tail -3 $O/fe_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "baseline_configs or near_threshold or bit_exact" -s > $O/parity_new.log 2>&1 || { echo "parity failed"; tail -30 $O/parity_new.log; exit 1; }
grep -E "passed|failed|flips" $O/parity_new.log | tail -3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
