#!/bin/bash
# Round 5: the new GPU tests (graph prepare, lazy ring, fused-scoring fallback) + the suites they
# touch, then the HealthRec leg at the driver's invocation (--steps 20 --warmup 5) and at 200/20,
# twice each, and the config-3 leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r5a}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_graph_prepare_gpu.py tests/test_rank_gpu.py tests/test_late_drain_gpu.py \
  tests/test_models_gpu.py tests/test_rowgrad_gpu.py "tests/test_wide_gpu.py" -k "not (CIKM or PRICAI) or not wide" -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests_$TAG.log 2>&1 || { grep -E "FAILED|ERROR|Error" $OUT/gpu_tests_$TAG.log | head; tail -30 $OUT/gpu_tests_$TAG.log; exit 1; }
tail -2 $OUT/gpu_tests_$TAG.log
HR="--no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval"
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 $HR > $OUT/hr20_${TAG}_$k.json 2> $OUT/hr20_${TAG}_$k.err \
    || { tail -20 $OUT/hr20_${TAG}_$k.err; exit 1; }
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 $HR > $OUT/hr200_${TAG}_$k.json 2> $OUT/hr200_${TAG}_$k.err \
    || { tail -20 $OUT/hr200_${TAG}_$k.err; exit 1; }
done
for f in $OUT/hr20_${TAG}_*.json $OUT/hr200_${TAG}_*.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d['timed_region'], d['epoch_sampling']['lazy_flush_ms_per_epoch'], d['epoch_sampling']['steps_ms_per_step'])" $f
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline --no-eval \
  > $OUT/c3_$TAG.json 2> $OUT/c3_$TAG.err || { tail -20 $OUT/c3_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config3_clussl_foodcom']; print(json.dumps({k: c[k] for k in c if k != 'cpu_baseline'}))" $OUT/c3_$TAG.json
