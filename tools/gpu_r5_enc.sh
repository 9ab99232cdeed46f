#!/bin/bash
# Round 5 encoder backward A/B: GPU encoder tests, then rocprofv3 kernel stats of the fused layer
# micro-benchmark (HealthRec shape) with the row-streaming vs the round-4 partial reduction, and the
# per-phase stamps of workgroup 0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r5e}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_encoder_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/enc_tests_$TAG.log 2>&1 || { tail -30 $OUT/enc_tests_$TAG.log; exit 1; }
tail -1 $OUT/enc_tests_$TAG.log
cd /tmp && export TMPDIR=/tmp
for m in 1 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/encprof_${TAG}_$m -o run -- python3 $R/tools/bench_encoder.py \
    --reduce-mode $m --no-torch --iters 30 > $OUT/enc_${TAG}_$m.json 2> $OUT/enc_${TAG}_$m.err || { tail -5 $OUT/enc_${TAG}_$m.err; exit 1; }
  f=$(find $OUT/encprof_${TAG}_$m -name "*kernel_stats.csv" | head -1)
  echo "mode $m"; grep -E "enc_|Name" "$f" | cut -d, -f1-8
done
timeout -k 10 120 python3 $R/tools/bench_encoder.py --phases --no-torch --iters 20 > $OUT/enc_${TAG}_phases.json 2>&1 || exit 1
tail -c 1500 $OUT/enc_${TAG}_phases.json
