#!/bin/bash
# InfoNCE A/B: parity tests on the working tree's library, then the SSL fwd+bwd graph replays with it
# and with ab/libfr_engine_${BASE:-ncehead}.so alternately, and a rocprofv3 kernel-stats pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-nce}
BASE=${BASE:-ncehead}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_wide_gpu.py tests/test_models_gpu.py -m gpu -x -q \
  -k "infonce or nce or dcor or PRICAI" --timeout 200 --timeout-method thread > $OUT/nce_tests_$TAG.log 2>&1 \
  || { grep -E "FAILED|Error|assert" $OUT/nce_tests_$TAG.log | head; tail -20 $OUT/nce_tests_$TAG.log; exit 1; }
tail -1 $OUT/nce_tests_$TAG.log
for k in 1 2; do
  timeout -k 10 120 python3 tools/profile_ssl.py 1 > $OUT/nce_${TAG}_new$k.json 2>&1 || { tail -5 $OUT/nce_${TAG}_new$k.json; exit 1; }
  echo "new: $(tail -1 $OUT/nce_${TAG}_new$k.json)"
  FR_ENGINE_LIB=$R/ab/libfr_engine_$BASE.so timeout -k 10 120 python3 tools/profile_ssl.py 1 > $OUT/nce_${TAG}_base$k.json 2>&1 || { tail -5 $OUT/nce_${TAG}_base$k.json; exit 1; }
  echo "base: $(tail -1 $OUT/nce_${TAG}_base$k.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_nce_$TAG -o run -- python3 $R/tools/profile_ssl.py \
  > $OUT/nce_prof_$TAG.log 2>&1 || { tail -5 $OUT/nce_prof_$TAG.log; exit 1; }
python3 - $(find $OUT/prof_nce_$TAG -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if "nce" in n:
        print("  ", n[:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
