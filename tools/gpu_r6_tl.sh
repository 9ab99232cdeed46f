#!/bin/bash
# (round 6) One HealthRec step's kernel timeline (TL_KS steps from the end, default 38 40 42: the last ~20 feed launches are the
# eager kernel pass) under rocprofv3 --kernel-trace for each "tag:ENV=V ..." spec.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  for kv in $envs; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tl_$tag -o run -- python3 $R/bench.py --steps 60 \
    --warmup 10 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval > $OUT/tl_$tag.json \
    2> $OUT/tl_$tag.err || { echo "$tag rocprof failed"; tail -20 $OUT/tl_$tag.err; exit 1; }
  for kv in $envs; do unset "${kv%%=*}"; done
  f=$(find $OUT/tl_$tag -name "*kernel_trace.csv" | head -1)
  for k in ${TL_KS:-38 40 42}; do
    python3 $R/tools/step_timeline.py "$f" $k > $OUT/step_timeline_${tag}_$k.txt && tail -1 $OUT/step_timeline_${tag}_$k.txt
  done
done
