#!/bin/bash
# rocprofv3 kernel trace of the world-1 data-parallel HealthRec step (FR_BENCH_DP1=1)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dp1}
OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
FR_BENCH_DP1=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 20 \
  --warmup 5 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err \
  || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
cut -c1-300 $OUT/bench_prof_$TAG.json
