#!/bin/bash
# GPU tests (optionally a subset): python -u pytest with per-test thread timeouts, log under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-t}
shift
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/gpu_tests_$TAG.log | tail -40
exit $rc
