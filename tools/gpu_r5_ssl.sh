#!/bin/bash
# Round 5 SSL kernels: the InfoNCE / dCor parity tests (kernel and CLUSSL fixtures), then the SSL fwd+bwd
# graph replays with the round-5 (1) and round-4 (2) MFMA InfoNCE kernels, twice each, and one
# rocprofv3 kernel-stats pass of the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r5s}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_wide_gpu.py tests/test_models_gpu.py -m gpu -x -q \
  -k "infonce or dcor or nce or PRICAI" --timeout 200 --timeout-method thread > $OUT/ssl_tests_$TAG.log 2>&1 \
  || { grep -E "FAILED|Error|assert" $OUT/ssl_tests_$TAG.log | head; tail -20 $OUT/ssl_tests_$TAG.log; exit 1; }
tail -1 $OUT/ssl_tests_$TAG.log
for mode in ${SSL_MODES:-1 2 1 2}; do
  timeout -k 10 120 python3 tools/profile_ssl.py $mode > $OUT/ssl_${TAG}_m$mode.json 2>&1 || { tail -5 $OUT/ssl_${TAG}_m$mode.json; exit 1; }
  echo "mode $mode: $(tail -1 $OUT/ssl_${TAG}_m$mode.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_ssl_$TAG -o run -- python3 $R/tools/profile_ssl.py \
  > $OUT/ssl_prof_$TAG.log 2>&1 || { tail -5 $OUT/ssl_prof_$TAG.log; exit 1; }
python3 - $(find $OUT/prof_ssl_$TAG -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if "nce" in n or "dcor" in n:
        print("  ", n[:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
