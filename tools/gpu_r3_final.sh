#!/bin/bash
# Full gate on HEAD: every -m gpu test, smoke(), the default bench line, the world-1 data-parallel leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-final}
mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests_$TAG.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -5 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 900 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cut -c1-400 $OUT/bench_$TAG.json
FR_BENCH_DP1=1 timeout -k 10 600 python bench.py --steps 100 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval \
  > $OUT/bench_dp1_$TAG.json 2> $OUT/bench_dp1_$TAG.err || { tail -20 $OUT/bench_dp1_$TAG.err; exit 1; }
cut -c1-300 $OUT/bench_dp1_$TAG.json
