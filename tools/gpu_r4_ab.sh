#!/bin/bash
# Round-4 A/B: encoder tests + phase stamps, then HealthRec legs (AB_STEPS steps) under env settings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-ab}
shift
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest ${R4_TESTS:-tests/test_encoder_gpu.py} -m gpu -q --timeout 200 --timeout-method thread \
  > $OUT/${TAG}_tests.log 2>&1; rc=$?; tail -2 $OUT/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_encoder.py --phases > $OUT/${TAG}_encb.json 2> $OUT/${TAG}_encb.err || exit 1
tail -c 1200 $OUT/${TAG}_encb.json; echo
AB_STEPS=${AB_STEPS:-300} bash tools/gpu_ab_lib.sh "$@"
