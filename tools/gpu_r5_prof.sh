#!/bin/bash
# rocprofv3 kernel stats of the driver's HealthRec invocation (HealthRec leg only) and the graphed
# steps' average kernel durations (tools/graph_kernel_avg.py), beside the line's in-graph stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r5p2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 20 \
  --warmup 5 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval > $OUT/prof_$TAG.json \
  2> $OUT/prof_$TAG.err || { tail -20 $OUT/prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/graph_kernel_avg.py "$f" 20 20 > $OUT/graph_kernel_avg_$TAG.json
python3 -c "import json,sys; g=json.load(open(sys.argv[1])); d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print('trace enc_bwd+reduce per call us', g.get('_encoder_bwd_call_us'), 'steps', g['_steps']); print('line', d['roofline']['avg_launch_ms'], d['roofline']['frac'])" $OUT/graph_kernel_avg_$TAG.json $OUT/prof_$TAG.json
for k in 26 27 28; do python3 $R/tools/step_timeline.py "$f" $((k+20)) > $OUT/step_timeline_${TAG}_$k.txt; done
tail -1 $OUT/step_timeline_${TAG}_26.txt
