#!/bin/bash
# Round 5, batch 2: the whole GPU suite, the SSL replays (fused InfoNCE launches = mode 1 vs the
# separate normalize / sum launches = mode 3), the config-3 leg, then HealthRec A/B specs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/b2_tests.log 2>&1 \
  || { grep -E "FAILED|Error|assert" $OUT/b2_tests.log | head -20; tail -30 $OUT/b2_tests.log; exit 1; }
tail -1 $OUT/b2_tests.log
for mode in 1 3 1 3; do
  timeout -k 10 120 python3 tools/profile_ssl.py $mode > $OUT/ssl_b2_m$mode.json 2>&1 || { tail -5 $OUT/ssl_b2_m$mode.json; exit 1; }
  echo "mode $mode: $(tail -1 $OUT/ssl_b2_m$mode.json)"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_ssl_b2 -o run -- \
  python3 $R/tools/profile_ssl.py > $OUT/ssl_prof_b2.log 2>&1) || { tail -5 $OUT/ssl_prof_b2.log; exit 1; }
python3 - $(find $OUT/prof_ssl_b2 -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if "nce" in n or "dcor" in n:
        print("  ", n[:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline --no-eval \
  > $OUT/b2_c3.json 2> $OUT/b2_c3.err || { tail -20 $OUT/b2_c3.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config3_clussl_foodcom']; print('c3', c['dcor']['ms_per_step'], c['infonce']['ms_per_step'], c.get('roofline'))" $OUT/b2_c3.json
AB_STEPS=300 bash tools/gpu_ab_lib.sh "$@"
