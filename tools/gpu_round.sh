#!/bin/bash
# One GPU session: smoke -> bench -> rocprofv3 kernel trace (stops at the first failure).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
STEPS=${2:-30}
mkdir -p $OUT
cd $R
echo "[smoke]" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
echo "[bench]" && timeout -k 10 600 python bench.py --steps $STEPS --warmup 10 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
echo "[rocprof]"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
find $OUT/prof_$TAG -name "*kernel_stats.csv" | head -3
exit 0
