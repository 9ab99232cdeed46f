#!/bin/bash
# HealthRec leg only: bench line (graphed step), then rocprofv3 --kernel-trace --stats of the same
# leg + the per-step kernel breakdown.  Usage: gpu_hr_quick.sh TAG [STEPS]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-hrq}
STEPS=${2:-50}
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py --steps $STEPS --warmup 10 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline \
  > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail -20 $OUT/bench_$TAG.err; exit 1; }
cut -c1-420 $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 20 \
  --warmup 5 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err \
  || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py "$f" 60 --steps 20 > $OUT/step_breakdown_$TAG.txt && head -30 $OUT/step_breakdown_$TAG.txt | cut -c1-150
exit 0
