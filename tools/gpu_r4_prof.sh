#!/bin/bash
# Round-4 profiling batch: HealthRec leg under rocprofv3 (kernel stats + one step's timeline), the
# config-3 leg under rocprofv3 (kernel stats), A/B of FR_PROJECTION_FIRST.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r4p}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 30 \
  --warmup 5 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval > $OUT/bench_prof_$TAG.json \
  2> $OUT/bench_prof_$TAG.err || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_timeline.py "$f" 3 > $OUT/step_timeline_$TAG.txt && tail -60 $OUT/step_timeline_$TAG.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/c3prof_$TAG -o run -- python3 $R/tools/profile_c3.py \
  > $OUT/c3_$TAG.json 2> $OUT/c3_$TAG.err || { echo c3 rocprof failed; tail -20 $OUT/c3_$TAG.err; exit 1; }
cut -c1-600 $OUT/c3_$TAG.json
cd $R
AB_STEPS=300 bash tools/gpu_ab_lib.sh ${TAG}_pf1:head:FR_PROJECTION_FIRST=1 ${TAG}_pf0:head ${TAG}_pf1b:head:FR_PROJECTION_FIRST=1 ${TAG}_pf0b:head
