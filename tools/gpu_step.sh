#!/bin/bash
# HealthRec step anatomy: bench (HealthRec leg only) under a rocprofv3 kernel trace -> per-step kernel
# breakdown; torch.profiler op table of the eager step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-step}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $OUT/trace_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 5 \
  --no-spmm-10m --no-config5 --no-cpu-baseline > $OUT/bench_trace_$TAG.json 2> $OUT/bench_trace_$TAG.err \
  || { echo trace failed; tail -20 $OUT/bench_trace_$TAG.err; exit 1; }
f=$(find $OUT/trace_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py "$f" 45 --steps 20 > $OUT/step_breakdown_$TAG.txt && head -46 $OUT/step_breakdown_$TAG.txt | cut -c1-170
cd $R
timeout -k 10 300 python3 tools/profile_step.py > $OUT/op_profile_$TAG.txt 2> $OUT/op_profile_$TAG.err || { echo profile failed; tail -20 $OUT/op_profile_$TAG.err; exit 1; }
exit 0
