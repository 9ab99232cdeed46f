#!/bin/bash
# Round-4: placement of the work beside the encoder forward on the HealthRec leg, after the row tests:
# the background slice start point (FR_SLICE_DEFER) and grid caps of the propagation / slice
# (FR_SPMM_GRID_CAP, FR_SLICE_GRID_CAP).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-sl}
mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_rowgrad_gpu.py -m gpu -q --timeout 200 --timeout-method thread \
  > $OUT/${TAG}_tests.log 2>&1; rc=$?; tail -2 $OUT/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
AB_STEPS=300 bash tools/gpu_ab_lib.sh ${TAG}_base:head ${TAG}_enc:head:FR_SLICE_DEFER=enc ${TAG}_head:head:FR_SLICE_DEFER=head \
  ${TAG}_sp64:head:FR_SPMM_GRID_CAP=64 ${TAG}_sp128:head:FR_SPMM_GRID_CAP=128 ${TAG}_sl32:head:FR_SLICE_GRID_CAP=32 \
  "${TAG}_sp64sl32:head:FR_SPMM_GRID_CAP=64 FR_SLICE_GRID_CAP=32" ${TAG}_base2:head ${TAG}_enc2:head:FR_SLICE_DEFER=enc
