#!/bin/bash
# config-3 tests + bench legs, then the config-3 leg under rocprofv3 (kernel stats + trace).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-c3p}
mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "views or weights or split or dcor or infonce" \
  --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; rc=$?; tail -3 $OUT/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_c3_ab.sh ${TAG}_a ${TAG}_b || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/c3prof_$TAG -o run -- python3 $R/tools/profile_c3.py \
  > $OUT/c3_$TAG.json 2> $OUT/c3_$TAG.err || { echo c3 rocprof failed; tail -20 $OUT/c3_$TAG.err; exit 1; }
f=$(find $OUT/c3prof_$TAG -name "*kernel_stats.csv" | head -1)
head -30 "$f" | cut -d, -f1-4 | cut -c1-150
