#!/bin/bash
# Encoder round-4 check: encoder / HealthRec / wide GPU tests, the encoder micro-benchmark (phase
# stamps), then the HealthRec leg (AB_STEPS steps, default 300).  Usage: gpu_r4_enc.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-enc}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest ${R4_TESTS:-tests} \
  -m gpu -q --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
rc=$?
tail -3 $OUT/${TAG}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_encoder.py --phases > $OUT/${TAG}_encb.json 2> $OUT/${TAG}_encb.err || exit 1
tail -c 1200 $OUT/${TAG}_encb.json; echo
AB_STEPS=${AB_STEPS:-300} bash tools/gpu_ab_lib.sh ${TAG}_hr1:head ${TAG}_hr2:head
