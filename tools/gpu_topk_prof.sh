#!/bin/bash
# rocprofv3 --kernel-trace --stats of the config-5 full-sort top-k (tools/bench_topk.py) -> gpurun_out/prof_topk_TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-a}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_topk_$TAG -o run -- python3 $R/tools/bench_topk.py \
  --only 20,1 --reps 3 > $OUT/topk_$TAG.log 2>&1 || { echo "topk failed"; tail -5 $OUT/topk_$TAG.log; exit 1; }
grep -v "^W\|^E20" $OUT/topk_$TAG.log | tail -3
cut -d, -f1-4 $(find $OUT/prof_topk_$TAG -name "*kernel_stats.csv") | cut -c1-150 | head -12
