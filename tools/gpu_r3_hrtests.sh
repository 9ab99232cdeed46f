#!/bin/bash
# HealthRec-path GPU tests, then A/B runs of the HealthRec leg: gpu_r3_hrtests.sh "tag:LIB:ENV" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 700 python -u -m pytest tests/test_models_gpu.py tests/test_wide_gpu.py tests/test_rowgrad_gpu.py tests/test_rccl_gpu.py \
  tests/test_multirank_gpu.py tests/test_projection_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/hr_tests.log 2>&1
rc=$?; tail -3 gpurun_out/hr_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_lib.sh "$@"
