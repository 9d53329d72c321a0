# On the GPU box: the on-the-fly Scharr probe (times + checksums) and its SQ
# instruction mix per wave (one --pmc pass).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
timeout -k 5 120 ./tools/lk_scharr_probe > $O/lk_scharr_probe.txt 2>&1 || { cat $O/lk_scharr_probe.txt; exit 1; }
cat $O/lk_scharr_probe.txt
rm -rf $O/lkp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU \
    SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d $O/lkp -o run --output-format csv -- ./tools/lk_scharr_probe > $O/lkp.log 2>&1 \
    || { tail -5 $O/lkp.log; exit 1; }
python3 - $O/lkp <<'P' | tee -a $O/lk_scharr_probe.txt
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "gather" if "gather" in r["Kernel_Name"] else "fly"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    w = d["SQ_WAVES"]
    print("per wave", k, " ".join("%s=%.0f" % (c.replace("SQ_", ""), v / w) for c, v in sorted(d.items()) if c != "SQ_WAVES"))
P
