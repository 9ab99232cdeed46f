#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, kernel trace only): the full-sort top-k call and the
# SSL fwd+bwd replays.  Per-kernel sums in gpurun_out/sqpmc_<name>.txt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
run() {
  name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc $CTR --kernel-trace -f csv -d $OUT/sqpmc_$name -o run -- "$@" > $OUT/sqpmc_$name.log 2>&1 \
    || { echo "$name failed"; tail -5 $OUT/sqpmc_$name.log; exit 1; }
  python3 - $(find $OUT/sqpmc_$name -name "*counter_collection.csv") > $OUT/sqpmc_$name.txt <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    calls = max(n[(k, c)] for c in d)
    print(k, "calls", calls, {c: round(v / calls) for c, v in sorted(d.items())})
PY
  cat $OUT/sqpmc_$name.txt | grep -E "topk|nce_bwd|nce_lse|dcor_bwd|dcor_tiles"
}
run topk python3 $R/tools/bench_topk.py --only 20,0 --reps 1
run ssl python3 $R/tools/profile_ssl.py
