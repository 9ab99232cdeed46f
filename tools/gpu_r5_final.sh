#!/bin/bash
# Round 5 evidence batch: the whole -m gpu suite, smoke(), the driver's bench invocation and the
# default bench line (all legs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r5z}
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1 \
  || { grep -E "FAILED|Error" $OUT/gpu_tests_$TAG.log | head; tail -20 $OUT/gpu_tests_$TAG.log; exit 1; }
tail -1 $OUT/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -2 $OUT/smoke_$TAG.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_$TAG.json 2> $OUT/bench_driver_$TAG.err \
  || { tail -20 $OUT/bench_driver_$TAG.err; exit 1; }
timeout -k 10 600 python -u bench.py > $OUT/bench_full_$TAG.json 2> $OUT/bench_full_$TAG.err || { tail -20 $OUT/bench_full_$TAG.err; exit 1; }
for f in $OUT/bench_driver_$TAG.json $OUT/bench_full_$TAG.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; c3=d['config3_clussl_foodcom']; c4=d['config4_10m']['spmm']; print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], 'c3', c3['dcor']['ms_per_step'], c3['infonce']['ms_per_step'], c3['roofline']['frac'], 'c4spmm', c4['frac'], c4.get('traffic_gbps'), 'topk', d['config5_10m_bf16']['full_sort_topk']['frac'])" $f
done
