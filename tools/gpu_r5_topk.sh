#!/bin/bash
# Round 5 top-k: the config-5 GPU tests (every APPEND shape on the sampled path), then each APPEND shape
# timed at the config-5 size (32,768 users x 1M items x d 256 bf16, k 20, no mask) and one rocprofv3
# kernel-stats pass of the chosen shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r5t}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_config5_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/topk_tests_$TAG.log 2>&1 || { grep -E "FAILED|Error|assert" $OUT/topk_tests_$TAG.log | head; tail -20 $OUT/topk_tests_$TAG.log; exit 1; }
tail -1 $OUT/topk_tests_$TAG.log
for sh in 0 1; do
  timeout -k 10 120 python3 tools/bench_topk.py --only 20,0 --reps 5 > $OUT/topk_${TAG}_s$sh.log 2>&1 || { tail -5 $OUT/topk_${TAG}_s$sh.log; exit 1; }
  echo "shape $sh: $(grep TFLOP $OUT/topk_${TAG}_s$sh.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_topk_$TAG -o run -- python3 $R/tools/bench_topk.py \
  --only 20,0 --reps 3 > $OUT/topk_prof_$TAG.log 2>&1 || { tail -5 $OUT/topk_prof_$TAG.log; exit 1; }
cut -d, -f1-4 $(find $OUT/prof_topk_$TAG -name "*kernel_stats.csv") | cut -c1-150 | head -8
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_ssl_$TAG -o run -- python3 $R/tools/profile_ssl.py \
  > $OUT/ssl_prof_$TAG.log 2>&1 || { tail -5 $OUT/ssl_prof_$TAG.log; exit 1; }
cut -d, -f1-4,6 $(find $OUT/prof_ssl_$TAG -name "*kernel_stats.csv") | cut -c1-150 | grep -E "nce|dcor|Name"
