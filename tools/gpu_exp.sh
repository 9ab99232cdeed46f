#!/bin/bash
# A/B experiments on the HealthRec leg: env toggles read by the engine (FR_EXP_*), 200 steps each.
mkdir -p gpurun_out
HR="--steps 200 --warmup 10 --no-config3 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline"
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py $HR > gpurun_out/exp_$tag.json 2> gpurun_out/exp_$tag.err || exit $?
  python -c "import json,sys;d=json.loads(open('gpurun_out/exp_$tag.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$tag', d['value'], d['ms_per_step'], {n:k[n]['avg_ms'] for n in k if n in ('adam','spmm_sparse','spmm_masked','spmm','encoder_bwd')})"
}
timeout -k 10 120 env FR_EXP_GBITS=0 python -u tools/diag/masked_spmm.py || exit $?
timeout -k 10 120 env FR_EXP_GBITS=1 python -u tools/diag/masked_spmm.py || exit $?
run base
run gbits FR_EXP_GBITS=1
run plain FR_EXP_ADAM=1
run bpc8 FR_EXP_ADAM_BPC=8
run bpc3 FR_EXP_ADAM_BPC=3
run base2
