#!/bin/bash
# GPU session for the fused encoder layer: parity tests -> HealthRec bench (fused) -> A/B (unfused).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-enc}
mkdir -p $OUT
cd $R
echo "[tests]"
timeout -k 10 400 python -u -m pytest tests/test_encoder_gpu.py tests/test_gpu_kernels.py -k "encoder" -x -v \
  --timeout 120 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 || { echo tests failed; tail -40 $OUT/tests_$TAG.log; exit 1; }
tail -3 $OUT/tests_$TAG.log
echo "[bench fused]"
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --no-spmm-10m --no-config5 --no-cpu-baseline \
  > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail -20 $OUT/bench_$TAG.err; exit 1; }
cut -c1-400 $OUT/bench_$TAG.json
echo "[bench unfused]"
FR_FUSED_ENCODER=0 timeout -k 10 400 python bench.py --steps 30 --warmup 10 --no-spmm-10m --no-config5 --no-cpu-baseline \
  > $OUT/bench_${TAG}_off.json 2> $OUT/bench_${TAG}_off.err || { echo bench failed; tail -20 $OUT/bench_${TAG}_off.err; exit 1; }
cut -c1-400 $OUT/bench_${TAG}_off.json
exit 0
