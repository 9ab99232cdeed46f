#!/bin/bash
# Fused encoder iteration: parity tests -> micro-benchmark -> rocprofv3 kernel stats of the micro-benchmark.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-enc}
mkdir -p $OUT
cd $R
echo "[tests]"
timeout -k 10 400 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/tests_$TAG.log 2>&1 || { echo tests failed; tail -40 $OUT/tests_$TAG.log; exit 1; }
tail -2 $OUT/tests_$TAG.log
echo "[micro]"
timeout -k 10 300 python tools/bench_encoder.py --phases > $OUT/micro_$TAG.json 2> $OUT/micro_$TAG.err || { echo micro failed; tail -20 $OUT/micro_$TAG.err; exit 1; }
cat $OUT/micro_$TAG.json
echo "[rocprof]"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/tools/bench_encoder.py \
  > $OUT/micro_prof_$TAG.json 2> $OUT/micro_prof_$TAG.err || { echo rocprof failed; tail -20 $OUT/micro_prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_stats.csv" | head -1)
head -12 "$f" | cut -c1-200
exit 0
