#!/bin/bash
# Round 6 encoder A/B on one box: for each library (ab/libfr_engine_NAME.so, or "cur" = the in-tree
# build) the fused layer micro-benchmark's per-phase stamps and rocprofv3 kernel stats.  Optionally the
# encoder GPU tests first (--tests), on the in-tree build.
#   tools/gpu_r6_encab.sh TAG [--tests] NAME...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; shift
mkdir -p $OUT
cd $R
if [ "$1" == "--tests" ]; then
  shift
  timeout -k 10 400 python -u -m pytest tests/test_encoder_gpu.py tests/test_dropout_model_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $OUT/encab_tests_$TAG.log 2>&1 || { tail -30 $OUT/encab_tests_$TAG.log; exit 1; }
  tail -1 $OUT/encab_tests_$TAG.log
fi
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for NAME in "$@"; do
  if [ "$NAME" == "cur" ]; then LIB=""; else LIB=$R/ab/libfr_engine_$NAME.so; fi
  FR_ENGINE_LIB=$LIB timeout -k 10 120 python3 $R/tools/bench_encoder.py --phases --no-torch --iters 20 \
    > $OUT/encab_${TAG}_${NAME}_ph$rep.json 2>&1 || { tail -5 $OUT/encab_${TAG}_${NAME}_ph$rep.json; exit 1; }
  FR_ENGINE_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/encab_${TAG}_${NAME}_$rep -o run -- \
    python3 $R/tools/bench_encoder.py --no-torch --iters 30 > /dev/null 2> $OUT/encab_${TAG}_${NAME}_$rep.err \
    || { tail -5 $OUT/encab_${TAG}_${NAME}_$rep.err; exit 1; }
  f=$(find $OUT/encab_${TAG}_${NAME}_$rep -name "*kernel_stats.csv" | head -1)
  echo "== $NAME rep $rep: $(python3 -c "
import json,sys; d=json.loads(open('$OUT/encab_${TAG}_${NAME}_ph$rep.json').read().strip().splitlines()[-1])
print('fwd', d['phases_cycles']['fwd']['total'], 'bwd', d['phases_cycles']['bwd']['total'])")"
  grep -E "enc_" "$f" | awk -F, '{printf "   %s avg %.1f us (min %.1f)\n", substr($1,1,40), $4/1000, $6/1000}'
done
done
