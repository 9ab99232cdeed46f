#!/bin/bash
# A/B runs of the HealthRec leg under env settings: gpu_exp.sh "tag:VAR=1 VAR2=x" "tag2:" ...
mkdir -p gpurun_out
HR="--steps 200 --warmup 10 --no-config3 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline"
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 150 python -u bench.py $HR > gpurun_out/exp_$tag.json 2> gpurun_out/exp_$tag.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/exp_$tag.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$tag', d['value'], d['ms_per_step'], d['epoch_sampling']['lazy_flush_ms_per_step'], {n:k[n]['avg_ms'] for n in k if not n.startswith('_')})"
done
