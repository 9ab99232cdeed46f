#!/bin/bash
# SQ counter passes over the fused encoder micro-benchmark (tools/bench_encoder.py): issue / stall /
# instruction-mix breakdown per kernel.  Each pass is its own rocprofv3 run (<= 8 SQ counters).
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out/pmc_enc${1:-}; mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -f csv -d $OUT -o p$n -- python3 $R/tools/bench_encoder.py --iters 3 \
    > $OUT/p$n.log 2>&1 || { echo "pass $n failed"; tail $OUT/p$n.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/p*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "enc_" not in r["Kernel_Name"]:
            continue
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k)
    for c, x in sorted(v.items()):
        print("   %-28s %.4g" % (c, x))
PY
