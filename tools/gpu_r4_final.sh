#!/bin/bash
# Round-4 evidence batch: rocprofv3 kernel trace + stats of the HealthRec leg (one step's timeline),
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) summarised per timing region into
# profiles/r4/pmc_traffic.json (read by bench.py's roofline.traffic), then the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r4f}
mkdir -p $OUT $R/profiles/r4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 40 \
  --warmup 8 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval > $OUT/bench_prof_$TAG.json \
  2> $OUT/bench_prof_$TAG.err || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_timeline.py "$f" 12 > $OUT/step_timeline_$TAG.txt && tail -3 $OUT/step_timeline_$TAG.txt
run() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $OUT/${name}_$TAG -o run -- "$@" > $OUT/${name}_$TAG.log 2>&1 || { echo "$name failed"; tail -5 $OUT/${name}_$TAG.log; exit 1; }
}
run pmc_fetch FETCH_SIZE python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmm-10m --no-config5 --no-config3 --no-config1 --no-eval
run pmc_write WRITE_SIZE python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmm-10m --no-config5 --no-config3 --no-config1 --no-eval
python3 $R/tools/pmc_regions.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_traffic_$TAG.json \
  "over bench.py --steps 5 --warmup 2 HealthRec leg (tools/gpu_r4_final.sh $TAG)" || exit 1
cp $OUT/pmc_traffic_$TAG.json $R/profiles/r4/pmc_traffic.json
cd $R
timeout -k 10 600 python -u bench.py > $OUT/bench_full_$TAG.json 2> $OUT/bench_full_$TAG.err || { echo bench failed; tail -20 $OUT/bench_full_$TAG.err; exit 1; }
tail -c 400 $OUT/bench_full_$TAG.json
