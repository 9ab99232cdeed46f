#!/bin/bash
# HealthRec gate: row-gradient parity tests, all -m gpu tests, the default bench line, then a
# rocprofv3 --kernel-trace --stats run of the HealthRec leg alone (its stats summary is the one the
# bench line's roofline kernel is checked against) + the per-step breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-hr}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_rowgrad_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/rowgrad_$TAG.log 2>&1 || { echo rowgrad failed; tail -30 $OUT/rowgrad_$TAG.log; exit 1; }
tail -1 $OUT/rowgrad_$TAG.log
bash tools/gpu_full.sh $TAG || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 20 \
  --warmup 5 --no-spmm-10m --no-config5 --no-cpu-baseline > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err \
  || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py "$f" 45 --steps 20 > $OUT/step_breakdown_$TAG.txt && head -12 $OUT/step_breakdown_$TAG.txt | cut -c1-150
exit 0
