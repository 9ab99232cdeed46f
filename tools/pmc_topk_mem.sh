#!/bin/bash
# Memory-side PMC pass over the fused top-k: DRAM fetch bytes and L2 hits / misses per kernel.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out/pmc_topk_mem; mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace -f csv -d $OUT -o m -- python3 $R/tools/bench_topk.py --only 20,1 --reps 1 > $OUT/m.log 2>&1 || { echo fail; tail $OUT/m.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace -f csv -d $OUT -o n -- python3 $R/tools/bench_topk.py --only 20,1 --reps 1 > $OUT/n.log 2>&1 || { echo fail; tail $OUT/n.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "topk" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: "%.4g" % x for c, x in v.items()})
PY
