#!/bin/bash
# Round 6 step A/B over environment settings on one box (the in-tree library): the HealthRec leg (300
# steps, eval / other configs off) for each "tag:ENV=V ..." spec, interleaved, REPS rounds.
#   tools/gpu_r6_envab.sh TAG REPS 'a:' 'b:FR_X=0' ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; REPS=$2; shift 2
mkdir -p $OUT
cd $R
HR="--steps 300 --warmup 10 --no-config3 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline --no-eval"
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 200 python -u bench.py $HR > $OUT/envab_${TAG}_${name}_$rep.json \
      2> $OUT/envab_${TAG}_${name}_$rep.err || { tail -5 $OUT/envab_${TAG}_${name}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/envab_${TAG}_${name}_$rep.json').read().strip().splitlines()[-1])
print('$name', $rep, d['value'], d['ms_per_step'], 'roof', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  done
done
