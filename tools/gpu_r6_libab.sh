#!/bin/bash
# Round 6 step A/B over engine libraries on one box: the HealthRec leg (300 steps, eval / other configs
# off) with each library (ab/libfr_engine_NAME.so, or "cur" = the in-tree build), interleaved, REPS
# rounds.  Prints value / ms per step per run.
#   tools/gpu_r6_libab.sh TAG REPS NAME...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; REPS=$2; shift 2
mkdir -p $OUT
cd $R
HR="--steps 300 --warmup 10 --no-config3 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline --no-eval"
for rep in $(seq 1 $REPS); do
  for NAME in "$@"; do
    if [ "$NAME" == "cur" ]; then LIB=""; else LIB=$R/ab/libfr_engine_$NAME.so; fi
    FR_ENGINE_LIB=$LIB timeout -k 10 200 python -u bench.py $HR > $OUT/libab_${TAG}_${NAME}_$rep.json \
      2> $OUT/libab_${TAG}_${NAME}_$rep.err || { tail -5 $OUT/libab_${TAG}_${NAME}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/libab_${TAG}_${NAME}_$rep.json').read().strip().splitlines()[-1])
k=d['kernels']; ig=k.get('_in_graph', {})
print('$NAME', $rep, d['value'], d['ms_per_step'], 'roof', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  done
done
