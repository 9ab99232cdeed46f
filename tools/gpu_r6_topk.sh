#!/bin/bash
# Round 6 top-k A/B: the config-5 GPU tests on the in-tree library, then the full-sort top-k at the
# config-5 size (32,768 users x 1M items x d 256 bf16, k 20) for each library, interleaved, REPS
# rounds, and one rocprofv3 kernel-stats pass per library.
#   tools/gpu_r6_topk.sh TAG REPS [--tests] NAME... (NAME "cur" = in-tree, else ab/libfr_engine_NAME.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; REPS=$2; shift 2
TESTS=0
if [ "$1" == "--tests" ]; then TESTS=1; shift; fi
mkdir -p $OUT
cd $R
if [ $TESTS == 1 ]; then
  timeout -k 10 500 python -u -m pytest tests/test_config5_gpu.py tests/test_config5_full_gpu.py -m gpu -x -q \
    --timeout 240 --timeout-method thread > $OUT/topk_tests_$TAG.log 2>&1 \
    || { grep -E "FAILED|Error|assert" $OUT/topk_tests_$TAG.log | head; tail -20 $OUT/topk_tests_$TAG.log; exit 1; }
  tail -1 $OUT/topk_tests_$TAG.log
fi
lib() { if [ "$1" == "cur" ]; then echo ""; else echo "FR_ENGINE_LIB=$R/ab/libfr_engine_$1.so"; fi; }
for rep in $(seq 1 $REPS); do
  for n in "$@"; do
    for v in "20,1" "20,0" "1,0"; do
      env $(lib $n) timeout -k 10 150 python3 tools/bench_topk.py --only $v --reps 5 > $OUT/topk_${TAG}_${n}_$rep.log 2>&1 \
        || { tail -5 $OUT/topk_${TAG}_${n}_$rep.log; exit 1; }
      echo "$n $rep: $(grep TFLOP $OUT/topk_${TAG}_${n}_$rep.log)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for n in "$@"; do
  env $(lib $n) timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_topk_${TAG}_$n -o run -- \
    python3 $R/tools/bench_topk.py --only 20,1 --reps 3 > $OUT/topk_prof_${TAG}_$n.log 2>&1 || { tail -5 $OUT/topk_prof_${TAG}_$n.log; exit 1; }
  echo "== $n"; cut -d, -f1-4 $(find $OUT/prof_topk_${TAG}_$n -name "*kernel_stats.csv") | cut -c1-150 | head -6
done
