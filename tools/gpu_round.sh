# Round-end style GPU session: parity suite, smoke, bench profile + PMC passes, bench line.
# Usage (on the box, from the repo root): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
B="python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-single"
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- $B > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
python tools/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv \
    profiles/pmc_summary.json --label "$TAG: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over '$B'" > $O/pmc_summary.txt 2>&1
cp profiles/pmc_summary.json $O/pmc_summary.json
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
for c in 1080p 4k; do timeout -k 10 400 python bench.py --config $c --seq 16 --steps 10 --warmup 2 --no-cpu-baseline --no-single > $O/bench_$c.log 2>&1 || { tail -5 $O/bench_$c.log; exit 1; }; tail -1 $O/bench_$c.log | cut -c1-400; done
timeout -k 10 600 bash tools/gpu_pmc_step.sh > $O/pmc_instructions.txt 2>&1 || { tail -5 $O/pmc_instructions.txt; exit 1; }
tail -20 $O/pmc_instructions.txt
