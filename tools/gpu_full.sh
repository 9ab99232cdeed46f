#!/bin/bash
# Full GPU gate: every -m gpu test, then the default bench line (HealthRec + config 4/5 legs + CPU baseline).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-full}
BENCH_ARGS=${2:-}
mkdir -p $OUT
cd $R
echo "[tests]"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests_$TAG.log 2>&1 || { echo tests failed; tail -40 $OUT/gpu_tests_$TAG.log; exit 1; }
tail -2 $OUT/gpu_tests_$TAG.log
echo "[bench]"
timeout -k 10 900 python bench.py $BENCH_ARGS > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err \
  || { echo bench failed; tail -20 $OUT/bench_$TAG.err; exit 1; }
cut -c1-600 $OUT/bench_$TAG.json
exit 0
