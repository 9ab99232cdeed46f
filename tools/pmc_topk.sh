#!/bin/bash
# SQ counter pass over the fused top-k (tools/bench_topk.py, one variant): stall / issue breakdown.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out/pmc_topk; mkdir -p $OUT
V=${1:-20,0}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -f csv -d $OUT -o sq -- python3 $R/tools/bench_topk.py --only $V --reps 1 > $OUT/sq.log 2>&1 || { echo fail; tail $OUT/sq.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/sq_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "topk" not in r["Kernel_Name"]:
        continue
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k)
    for c, x in sorted(v.items()):
        print("   %-28s %.4g" % (c, x))
PY
