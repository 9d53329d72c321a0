# LK kernel A/B between library builds (standalone, 128k features of one KITTI
# frame pair): rocprofv3 kernel time and the SQ counters (VALU, LDS, bank
# conflicts, waves) per build.
#   bash tools/lkcmp.sh libA.so libB.so ...   (names under svo_amd/lib)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
MB="python tools/microbench.py lk --points 128000 --reps 5"
for lib in "$@"; do
    T=/tmp/lkc_$lib
    SVO_GPU_LIB=$PWD/svo_amd/lib/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d ${T}_k -o run \
        --output-format csv -- $MB > ${T}.log 2>&1 || { echo "FAILED $lib trace"; tail -20 ${T}.log; exit 1; }
    SVO_GPU_LIB=$PWD/svo_amd/lib/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d ${T}_p -o run \
        --output-format csv -- $MB >> ${T}.log 2>&1 || { echo "FAILED $lib pmc"; tail -20 ${T}.log; exit 1; }
    python3 - $T $lib <<'P'
import csv, glob, sys, collections
T, lib = sys.argv[1], sys.argv[2]
dur = []
for f in glob.glob(T + '_k/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']:
            dur.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
agg = collections.defaultdict(float)
for f in glob.glob(T + '_p/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'lk_multi' in r['Kernel_Name']:
            agg[r['Counter_Name']] += float(r['Counter_Value'])
w = agg.get('SQ_WAVES', 1)
print(f"{lib}: lk_multi us {sorted(round(d, 1) for d in dur)} | per wave: " +
      ' '.join(f"{k.replace('SQ_', '')}={v / w:.0f}" for k, v in sorted(agg.items()) if k != 'SQ_WAVES'))
P
done
