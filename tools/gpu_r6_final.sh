#!/bin/bash
# Round 6 evidence batch.  Part "tests": the whole -m gpu suite and smoke().  Part "bench": the
# HealthRec leg's rocprofv3 kernel stats + graphed step timeline and its per-region PMC bytes
# (FETCH_SIZE / WRITE_SIZE in separate passes -> profiles/r6/pmc_traffic.json, read by bench.py's
# roofline `traffic`; copied into gpurun_out too), then the driver's bench invocation and the default
# bench line (all legs).
#   tools/gpu_r6_final.sh TAG tests|bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r6z}; PART=${2:-tests}
mkdir -p $OUT $R/profiles/r6
cd $R
if [ "$PART" == "tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1 \
    || { grep -E "FAILED|Error" $OUT/gpu_tests_$TAG.log | head; tail -20 $OUT/gpu_tests_$TAG.log; exit 1; }
  tail -1 $OUT/gpu_tests_$TAG.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -20 $OUT/smoke_$TAG.log; exit 1; }
  tail -2 $OUT/smoke_$TAG.log
  exit 0
fi
HR="--no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --gpus 1 --steps 20 \
  --warmup 5 $HR > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
for k in 10 12 14; do python3 $R/tools/step_timeline.py "$f" $k > $OUT/healthrec_step_timeline_${TAG}_$k.txt && tail -1 $OUT/healthrec_step_timeline_${TAG}_$k.txt; done
pmc() {  # name counter
  timeout -s KILL 240 rocprofv3 --pmc $2 --kernel-trace -f csv -d $OUT/${1}_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 2 $HR \
    > $OUT/${1}_$TAG.log 2>&1 || { echo "$1 failed"; tail -5 $OUT/${1}_$TAG.log; return 1; }
}
pmc pmc_fetch FETCH_SIZE || exit 1
pmc pmc_write WRITE_SIZE || exit 1
python3 $R/tools/pmc_regions.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $R/profiles/r6/pmc_traffic.json \
  "over bench.py --steps 5 --warmup 2 HealthRec leg (tools/gpu_r6_final.sh $TAG bench)" || exit 1
cp $R/profiles/r6/pmc_traffic.json $OUT/pmc_traffic_$TAG.json
cd $R
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_$TAG.json 2> $OUT/bench_driver_$TAG.err \
  || { tail -20 $OUT/bench_driver_$TAG.err; exit 1; }
timeout -k 10 700 python -u bench.py > $OUT/bench_full_$TAG.json 2> $OUT/bench_full_$TAG.err || { tail -20 $OUT/bench_full_$TAG.err; exit 1; }
for f in $OUT/bench_driver_$TAG.json $OUT/bench_full_$TAG.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; c3=d['config3_clussl_foodcom']; c4=d['config4_10m']['spmm']; print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['traffic'], 'c3', c3['dcor']['ms_per_step'], c3['infonce']['ms_per_step'], c3['dcor_fwd_bwd_ms'], 'c4spmm', c4['frac'], 'topk', d['config5_10m_bf16']['full_sort_topk']['frac'], d['config5_10m_bf16']['full_sort_topk']['avg_call_ms'])" $f
done
