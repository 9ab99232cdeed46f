#!/bin/bash
# Top-k clock / pipe pass: GRBM_GUI_ACTIVE (GPU clocks while busy) against the kernel trace's
# durations gives the effective clock; SQ_BUSY_CYCLES / MFMA busy / LDS activity of the same calls.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; OUT=$R/gpurun_out/pmc_topk_clk; mkdir -p $OUT
V=${1:-20,1}
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES --kernel-trace -f csv -d $OUT -o clk -- python3 $R/tools/bench_topk.py --only $V --reps 1 \
  > $OUT/clk.log 2>&1 || { echo fail; tail $OUT/clk.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/clk_counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
per = collections.defaultdict(dict)
for r in rows:
    if "topk_score_kernel<unsigned short, 256, 1, 1" not in r["Kernel_Name"]:
        continue
    key = r.get("Dispatch_Id") or r.get("Correlation_Id")
    per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k in ("Start_Timestamp", "End_Timestamp"):
        if k in r: per[key][k] = int(r[k])
for k, v in per.items():
    dur = (v.get("End_Timestamp", 0) - v.get("Start_Timestamp", 0)) / 1e3
    print(k, "dur_us", dur, {c: x for c, x in sorted(v.items()) if "Timestamp" not in c},
          "clk_GHz(GRBM/dur)", round(v.get("GRBM_GUI_ACTIVE", 0) / (dur * 1e3), 3) if dur > 0 else None)
PY
