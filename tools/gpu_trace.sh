# One steady-state step's GPU timeline (kernel + copy trace) and the host trace.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=/tmp/svo_trace
SVO_FE_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $T -o run --output-format csv -- python bench.py --steps ${1:-12} --warmup 3 --seq 64 --no-cpu-baseline --no-single ${2:-} > $T.log 2>&1 || { tail -5 $T.log; exit 1; }
python tools/timeline.py $T > gpurun_out/timeline.txt
grep "fe t=" $T.log | tail -14 > gpurun_out/hosttrace.txt
tail -1 $T.log | cut -c1-200 >> gpurun_out/hosttrace.txt
