#!/bin/bash
# Round-4 HealthRec step changes: tests (modal head, wide graphed / unrolled, rows, models), then the
# HealthRec leg A/B: unroll 4 vs 1 (config cuda_graph_unroll), modal head finalize in the forward's
# last block vs its own launch (FR_HEAD_TICKET).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-hr}
mkdir -p $OUT; cd $R
timeout -k 10 500 python -u -m pytest tests/test_modal_head_gpu.py tests/test_wide_gpu.py tests/test_rowgrad_gpu.py \
  tests/test_models_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
rc=$?; tail -3 $OUT/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
run() {  # tag env config_json
  env $2 timeout -k 10 300 python bench.py --steps 300 --warmup 10 --no-spmm-10m --no-config3 --no-config5 --no-config1 \
    --no-cpu-baseline --no-eval --config-json "$3" > $OUT/ab_$1.json 2> $OUT/ab_$1.err || { echo "$1 failed"; tail -5 $OUT/ab_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['config'].get('graph_steps_per_replay'))" $OUT/ab_$1.json $1
}
run ${TAG}_u4 "" '{}'
run ${TAG}_u1 "" '{"cuda_graph_unroll": 1}'
run ${TAG}_u4nt "FR_HEAD_TICKET=0" '{}'
run ${TAG}_u4b "" '{}'
run ${TAG}_u1b "" '{"cuda_graph_unroll": 1}'
run ${TAG}_u4ntb "FR_HEAD_TICKET=0" '{}'
