#!/bin/bash
# The band LIST kernel at configs[4] against the XCD item-block size
# (kItemBlock = 32 row tiles, the shipped value, vs 8 / 16 / 64): the kernel's
# average dispatch time (rocprofv3 --kernel-trace --stats) and its L2 hit rate
# (one --pmc pass: TCC_HIT_sum, TCC_MISS_sum), per library.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05ib
mkdir -p $O
CMD="python bench.py --genomes 10000 --sketch 10000 --steps 1 --warmup 0 --check 0 --cpu-baseline 0"
for V in default ib8 ib16 ib64 default; do
  LIBV=""; [ $V != default ] && LIBV=drep_amd/lib_ab/$V/libdrephip.so
  tag=$V.$RANDOM
  env ${LIBV:+DREPHIP_LIB=$LIBV} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${tag}_trace -o t -- $CMD > $O/${tag}_trace.log 2>&1 || { echo "$V trace failed"; tail -5 $O/${tag}_trace.log; exit 1; }
  env ${LIBV:+DREPHIP_LIB=$LIBV} timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/${tag}_p1 -o pmc -- $CMD > $O/${tag}_p1.log 2>&1 || { echo "$V pmc failed"; tail -5 $O/${tag}_p1.log; exit 1; }
  python3 - $O $tag $V <<'PY' | tee -a $O/summary.txt
import csv, glob, os, sys, collections
d, tag, v = sys.argv[1:4]
st = glob.glob(os.path.join(d, tag + "_trace", "**", "*kernel_stats.csv"), recursive=True)[0]
ms = [float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(st)) if "k_allpairs_band" in r["Name"]]
agg = collections.defaultdict(float)
for f in glob.glob(os.path.join(d, tag + "_p1", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_allpairs_band" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
h, m = agg.get("TCC_HIT_sum", 0), agg.get("TCC_MISS_sum", 0)
print("%-8s band kernel avg %.3f ms, L2 hit %.3f" % (v, ms[0] if ms else -1, h / max(1.0, h + m)))
PY
  rm -rf $O/${tag}_trace $O/${tag}_p1
done
