#!/bin/bash
# Round-4: config-3 SSL kernels, MFMA vs VALU Gram tiles (bench legs + rocprofv3 kernel stats of each),
# then the HealthRec leg's kernel trace / one step's timeline with the current defaults.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r4c}
mkdir -p $OUT
bash $R/tools/gpu_c3_ab.sh ${TAG}_mfma ${TAG}_valu:FR_SSL_MFMA=0 ${TAG}_mfma2 ${TAG}_valu2:FR_SSL_MFMA=0 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  FR_SSL_MFMA=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/c3prof_${TAG}_$v -o run -- \
    python3 $R/tools/profile_c3.py > $OUT/c3_${TAG}_$v.json 2> $OUT/c3_${TAG}_$v.err || { echo c3 rocprof failed; tail -20 $OUT/c3_${TAG}_$v.err; exit 1; }
  f=$(find $OUT/c3prof_${TAG}_$v -name "*kernel_stats.csv" | head -1)
  head -14 "$f" | cut -d, -f1-8
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 30 \
  --warmup 5 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval > $OUT/bench_prof_$TAG.json \
  2> $OUT/bench_prof_$TAG.err || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_timeline.py "$f" 3 > $OUT/step_timeline_$TAG.txt && tail -70 $OUT/step_timeline_$TAG.txt
