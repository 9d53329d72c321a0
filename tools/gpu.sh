# One driver for every GPU-box session (run from the repo root on the box):
#
#   bash tools/gpu.sh MODE [ARGS...] [-- MODE [ARGS...] ...]
#
#   tests [PYTEST_ARGS]     pytest -m gpu (default: the whole suite)
#   smoke                   __graft_entry__.smoke()
#   bench [BENCH_ARGS]      one bench.py line (default: the driver's defaults)
#   fe                      frontend + new-parity tests, short bench
#   trace [STEPS]           one steady step's GPU timeline + host trace
#   prof TAG [BENCH_ARGS]   rocprofv3 --kernel-trace --stats of a bench run
#   pmc TAG CONFIG [SEQ]    FETCH_SIZE / WRITE_SIZE passes of a bench run of CONFIG,
#                           folded into profiles/pmc_summary.json (configs[CONFIG])
#   mix TAG [BENCH_ARGS]    SQ instruction mix per wave of every step kernel
#                           (mix TAG --cmd CMD..: of any command's kernels)
#   lksplit                 LK VALU / time with the iteration cap at 1, 2, 50
#   lkab "V1 V2 .."         standalone LK kernel time per SVO_LK_VARIANT (or $LKAB_VAR) value
#   lkmem [LIB ..]          LK memory-pipeline + issue counters (TA, TCP, SQ), per library build
#   ab VAR "V1 V2" [RUNS]   bench A/B of an environment switch
#   abcfg VAR "V1 V2"       the same A/B at the 1080p, 4K and KITTI configs
#   round1 TAG / round2 TAG  the round records: tests, smoke, driver bench + rocprof / PMC, mix, 1080p + 4K
#
# Every GPU step has its own time limit; the first failure ends the session.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
BQ="python bench.py --steps ${AB_STEPS:-20} --warmup 5 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order --no-forward --no-orb --no-stream ${AB_ARGS:-}"

fail() { echo "FAILED: $1"; [ -n "$2" ] && tail -30 "$2"; exit 1; }

run_tests() {
    local args="${*:-tests}"
    timeout -k 10 900 python -u -m pytest $args -m gpu -x -v --timeout 150 --timeout-method thread \
        -p no:cacheprovider > $O/gpu_tests.log 2>&1 || fail tests $O/gpu_tests.log
    tail -1 $O/gpu_tests.log
}

run_smoke() {
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
    cat $O/smoke.log
}

run_bench() {
    local tag=$1; shift
    timeout -k 10 600 python bench.py "$@" > $O/bench_$tag.log 2>&1 || fail bench $O/bench_$tag.log
    tail -1 $O/bench_$tag.log | cut -c1-1500
}

run_fe() {
    timeout -k 10 600 python -u -m pytest tests/test_frontend_gpu.py tests/test_ingest.py -x -v --timeout 300 \
        --timeout-method thread -p no:cacheprovider -m gpu > $O/fe_tests.log 2>&1 || fail fe-tests $O/fe_tests.log
    tail -1 $O/fe_tests.log
    run_bench quick --steps 20 --warmup 5 --no-cpu-baseline
}

run_trace() {
    local T=/tmp/svo_trace
    local steps=${1:-12}; shift
    SVO_FE_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $T -o run --output-format csv -- \
        python bench.py --steps $steps --warmup 3 --seq 64 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order --no-forward --no-orb --no-stream "$@" \
        > $T.log 2>&1 || fail trace $T.log
    python tools/timeline.py $T > $O/timeline.txt
    grep "fe t=\|fe post t=" $T.log | tail -24 > $O/hosttrace.txt
    cat $O/timeline.txt $O/hosttrace.txt
}

run_prof() {
    local tag=$1; shift
    local args="${*:---steps 50 --warmup 10 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order --no-forward --no-orb --no-stream}"
    rm -rf $O/prof_$tag
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- \
        python bench.py $args > $O/prof_$tag.log 2>&1 || fail prof $O/prof_$tag.log
    tail -1 $O/prof_$tag.log | cut -c1-600
    python - $O/prof_$tag <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
P
}

run_pmc() {
    local tag=$1 cfg=$2 seq=${3:-128}
    local B="python bench.py --config $cfg --seq $seq --steps 10 --warmup 3 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order --no-forward --no-orb --no-stream"
    rm -rf $O/pmc_fetch_$cfg $O/pmc_write_$cfg
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$cfg -o run --output-format csv -- $B \
        > $O/pmc_fetch_$cfg.log 2>&1 || fail pmc-fetch $O/pmc_fetch_$cfg.log
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$cfg -o run --output-format csv -- $B \
        > $O/pmc_write_$cfg.log 2>&1 || fail pmc-write $O/pmc_write_$cfg.log
    python tools/pmc_summary.py $(find $O/pmc_fetch_$cfg -name "*counter_collection.csv" | head -1) \
        $(find $O/pmc_write_$cfg -name "*counter_collection.csv" | head -1) profiles/pmc_summary.json \
        --config $cfg --label "$tag: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over '$B'" || fail pmc-summary
    cp profiles/pmc_summary.json $O/pmc_summary.json
    rm -rf $O/pmc_fetch_$cfg $O/pmc_write_$cfg
}

run_mix() {
    local tag=$1; shift
    local B="python bench.py ${*:---seq 256 --steps 8 --warmup 2 --no-cpu-baseline --no-single --no-bucketed --no-opencv-order --no-forward --no-orb --no-stream}"
    [ "$1" = "--cmd" ] && { shift; B="$*"; }
    timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM -d /tmp/ps1 -o run --output-format csv -- $B > $O/mix.log 2>&1 || fail mix1 $O/mix.log
    timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS \
        SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d /tmp/ps2 -o run --output-format csv \
        -- $B >> $O/mix.log 2>&1 || fail mix2 $O/mix.log
    MIX_CMD="$B" MIX_JSON=$O/valu_$tag.json python - > $O/mix_$tag.txt <<'P'
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob('/tmp/ps[12]/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r'([a-z_0-9]+_kernel(<[^(]*>)?)', r['Kernel_Name'])
        if not m: continue
        k = m.group(1)
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add((f, r['Dispatch_Id']))
import json, os
summ = {}
for k, d in agg.items():
    n = len(disp[k]) / 2
    w = d.get('SQ_WAVES', 1)
    print(f"{k:40s} disp {n:5.0f} waves/disp {w/n:9.0f} | per wave: " + ' '.join(f"{c.replace('SQ_','')}={v/w:.0f}" for c, v in sorted(d.items()) if c != 'SQ_WAVES'))
    summ[k] = {"dispatches": n, "waves_per_dispatch": round(w / n, 1),
               "valu_per_dispatch": round(d.get('SQ_INSTS_VALU', 0) / n), "valu_per_wave": round(d.get('SQ_INSTS_VALU', 0) / w, 1)}
json.dump({"source": "SQ_INSTS_VALU / SQ_WAVES (rocprofv3 --pmc) of: " + os.environ.get("MIX_CMD", ""), "kernels": summ},
          open(os.environ["MIX_JSON"], "w"), indent=1)
P
    cat $O/mix_$tag.txt
    rm -rf /tmp/ps1 /tmp/ps2
}

run_lksplit() {
    for c in 1 2 50; do local T=/tmp/lks_$c
        timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
            -d $T -o run --output-format csv -- python tools/microbench.py lk --points 128000 --reps 2 --count $c \
            > $T.log 2>&1 || fail lksplit-pmc $T.log
        timeout -k 10 90 rocprofv3 --kernel-trace --stats -d ${T}k -o run --output-format csv -- \
            python tools/microbench.py lk --points 128000 --reps 3 --count $c >> $T.log 2>&1 || fail lksplit-time $T.log
        python - $T $c <<'P'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + '/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']: agg[r['Counter_Name']] += float(r['Counter_Value'])
dur = []
for f in glob.glob(sys.argv[1] + 'k/**/run_kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']: dur.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
print('count', sys.argv[2], 'us', [round(d, 1) for d in dur], ' '.join(f"{k}={v/2/128000*4:.0f}/wave" for k, v in sorted(agg.items())))
P
    done
}

run_lkab() {
    for v in ${1:-41}; do
        local T=/tmp/lkab_$(basename "$v")
        ( export "${LKAB_VAR:-SVO_LK_VARIANT}=$v"
          timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $T -o run --output-format csv -- \
            python tools/microbench.py lk --points 128000 --reps 5 > $T.log 2>&1 ) || fail lkab $T.log
        echo "== ${LKAB_VAR:-SVO_LK_VARIANT}=$v"
        python3 - $T <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'lk_multi' in r['Name'] or 'lk_fast' in r['Name'] or 'lk_dual' in r['Name']:
        print(r['Name'][40:110], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), round(float(r['MinNs']) / 1e3, 1))
P
    done
}

run_lkmem() {
    local MB="python tools/microbench.py lk --points 128000 --reps 2"
    for lib in ${@:-libsvo_gpu.so}; do
        local i=0
        for set in "TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
                   "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
                   "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
            i=$((i + 1))
            local T=/tmp/lkm_${lib}_$i
            SVO_GPU_LIB=$PWD/svo_amd/lib/$lib timeout -s KILL 90 rocprofv3 --pmc $set -d $T -o run --output-format csv -- $MB \
                > $T.log 2>&1 || fail "lkmem pass $i" $T.log
        done
        echo "== $lib"
        python3 - $lib <<'P'
import csv, glob, sys, collections
lib = sys.argv[1]
agg = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob(f'/tmp/lkm_{lib}_*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']:
            agg[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
w = agg.get('SQ_WAVES', 1)
for k in sorted(agg):
    print(f"  {k:40s} per dispatch {agg[k] / n[k]:14.0f}   per wave {agg[k] / w:10.1f}")
P
    done
}

run_ab() {
    local var=$1 vals=$2 runs=${3:-2}
    for r in $(seq $runs); do for v in $vals; do
        env $var=$v timeout -k 10 200 $BQ > $O/ab.log 2>&1 || fail ab $O/ab.log
        python -c "
import json; d=json.loads(open('$O/ab.log').read().strip().splitlines()[-1]); p=d['phase_ms_per_step']
sm=d.get('step_ms', {})
print('$var=$v', d['value'], d['ms_per_step'], 'median', sm.get('median'), 'p90', sm.get('p90'), 'lk', p['lk'], 'pyr', p['pyramid'],
      'fast_us', d['roofline_fast']['avg_launch_us'], d['roofline_fast']['frac'], 'pyr_us', d['roofline_pyramid']['avg_launch_us'], d['roofline_pyramid']['frac'])"
    done; done
}

run_abcfg() {
    local var=$1 vals=$2
    for cfg in 1080p 4k kitti; do
        local seq=16
        [ $cfg = kitti ] && seq=64
        for v in $vals; do
            env $var=$v timeout -k 10 200 python bench.py --config $cfg --seq $seq --steps 20 --warmup 5 --no-cpu-baseline \
                --no-single --no-bucketed --no-opencv-order --no-forward --no-orb --no-stream > $O/abc.log 2>&1 || fail abcfg $O/abc.log
            python -c "
import json; d=json.loads(open('$O/abc.log').read().strip().splitlines()[-1]); p=d['phase_ms_per_step']
print('$cfg $var=$v', d['value'], d['ms_per_step'], 'lk', p['lk'], 'stereo', p['stereo_lk'])"
        done
    done
}

# the round's records in two sessions (each fits one gpurun call): round1 = tests, smoke,
# the driver's bench command and its rocprof; round2 = PMC passes (3 configs), mix, the
# 1080p (64 sequences) and 4K (32) bench lines
run_round1() {
    local tag=$1
    run_tests
    run_smoke
    run_bench "${tag}_driver" --gpus 1 --steps 20 --warmup 5
    run_prof "$tag" --gpus 1 --steps 20 --warmup 5
}
run_round2() {
    local tag=$1
    run_pmc "$tag" kitti 256
    run_pmc "$tag" 1080p 64
    run_pmc "$tag" 4k 32
    run_mix "$tag"
    run_bench "${tag}_1080p" --config 1080p --seq 64 --steps 20 --warmup 5 --no-cpu-baseline
    run_bench "${tag}_4k" --config 4k --seq 32 --steps 20 --warmup 5 --no-cpu-baseline
}

while [ $# -gt 0 ]; do
    mode=$1; shift
    args=()
    while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done
    [ "$1" = "--" ] && shift
    case $mode in
        tests) run_tests "${args[@]}" ;;
        smoke) run_smoke ;;
        bench) run_bench main "${args[@]}" ;;
        fe) run_fe ;;
        trace) run_trace "${args[@]}" ;;
        prof) run_prof "${args[@]}" ;;
        pmc) run_pmc "${args[@]}" ;;
        mix) run_mix "${args[@]}" ;;
        lksplit) run_lksplit ;;
        lkab) run_lkab "${args[@]}" ;;
        lkmem) run_lkmem "${args[@]}" ;;
        ab) run_ab "${args[@]}" ;;
        abcfg) run_abcfg "${args[@]}" ;;
        round1) run_round1 "${args[@]}" ;;
        round2) run_round2 "${args[@]}" ;;
        *) fail "unknown mode $mode" ;;
    esac
done
