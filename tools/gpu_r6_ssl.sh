#!/bin/bash
# Round 6 SSL A/B: the InfoNCE / dCor parity tests (kernel and CLUSSL fixtures) on the in-tree
# library, then the SSL fwd+bwd graph replays (tools/profile_ssl.py) per library, interleaved, REPS
# rounds, and one rocprofv3 kernel-stats pass per library.
#   tools/gpu_r6_ssl.sh TAG REPS NAME...   (NAME "cur" = in-tree, else ab/libfr_engine_NAME.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; REPS=$2; shift 2
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_wide_gpu.py tests/test_models_gpu.py -m gpu -x -q \
  -k "infonce or dcor or nce or PRICAI" --timeout 200 --timeout-method thread > $OUT/ssl_tests_$TAG.log 2>&1 \
  || { grep -E "FAILED|Error|assert" $OUT/ssl_tests_$TAG.log | head; tail -20 $OUT/ssl_tests_$TAG.log; exit 1; }
tail -1 $OUT/ssl_tests_$TAG.log
lib() { if [ "$1" == "cur" ]; then echo ""; else echo "FR_ENGINE_LIB=$R/ab/libfr_engine_$1.so"; fi; }
for rep in $(seq 1 $REPS); do
  for n in "$@"; do
    env $(lib $n) timeout -k 10 120 python3 tools/profile_ssl.py > $OUT/ssl_${TAG}_${n}_$rep.json 2>&1 \
      || { tail -5 $OUT/ssl_${TAG}_${n}_$rep.json; exit 1; }
    echo "$n $rep: $(tail -1 $OUT/ssl_${TAG}_${n}_$rep.json)"
  done
done
cd /tmp && export TMPDIR=/tmp
for n in "$@"; do
  env $(lib $n) timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_ssl_${TAG}_$n -o run -- \
    python3 $R/tools/profile_ssl.py > $OUT/ssl_prof_${TAG}_$n.log 2>&1 || { tail -5 $OUT/ssl_prof_${TAG}_$n.log; exit 1; }
  echo "== $n"
  python3 - $(find $OUT/prof_ssl_${TAG}_$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if "nce" in n or "dcor" in n or "Fill" in n:
        print("  ", n[:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
