#!/bin/bash
# Round-3 profiling batch: HealthRec leg (bench line, rocprofv3 stats, step breakdown), the config-4
# single vs sharded P=1 step under rocprofv3 --kernel-trace --stats (csv), then the PMC traffic
# passes over HEAD's kernels.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r3a}
mkdir -p $OUT
cd $R
bash tools/gpu_hr_quick.sh $TAG 50 || exit 1
cd /tmp && export TMPDIR=/tmp
for m in single sharded; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/c4prof_${m}_$TAG -o run -- python3 $R/tools/profile_c4.py \
    --mode $m --batch 8192 --steps 3 > $OUT/c4_${m}_$TAG.log 2>&1 || { echo "c4 $m failed"; tail -5 $OUT/c4_${m}_$TAG.log; exit 1; }
  grep ms_per_step $OUT/c4_${m}_$TAG.log
done
bash $R/tools/gpu_pmc_r3.sh $TAG || exit 1
echo ok
