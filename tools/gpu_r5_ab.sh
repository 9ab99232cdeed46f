#!/bin/bash
# Round 5 A/B: named GPU test files first (comma list, or "-"), then gpu_ab_lib.sh specs, alternating.
#   gpu_r5_ab.sh "tests/test_late_drain_gpu.py,tests/test_models_gpu.py" "a1:head:FR_X=1" "a0:head:FR_X=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
T=$1; shift
if [ "$T" != "-" ]; then
  timeout -k 10 600 python -u -m pytest ${T//,/ } -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/ab_tests.log 2>&1 \
    || { grep -E "FAILED|Error" $OUT/ab_tests.log | head; tail -20 $OUT/ab_tests.log; exit 1; }
  tail -1 $OUT/ab_tests.log
fi
AB_STEPS=${AB_STEPS:-300} bash tools/gpu_ab_lib.sh "$@"
