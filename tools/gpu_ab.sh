#!/bin/bash
# A/B runs of the HealthRec leg with extra config keys: gpu_ab.sh 'tag=JSON' ...  (200 steps each)
mkdir -p gpurun_out
HR="--steps 200 --warmup 10 --no-config3 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline"
for spec in "$@"; do
  tag=${spec%%=*}; js=${spec#*=}
  timeout -k 10 150 python -u bench.py $HR --config-json "$js" > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]);k=d['kernels'];e=d['epoch_sampling'];print('$tag', d['value'], d['ms_per_step'], e['steps_ms_per_step'], e['lazy_flush_ms_per_epoch'], {n:k[n]['avg_ms'] for n in k if n.startswith('adam')})"
done
