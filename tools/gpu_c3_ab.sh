#!/bin/bash
# CLUSSL tests, then the config-3 leg under environment settings: gpu_c3_ab.sh "tag:ENV=V ..." ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_wide_gpu.py -x -q --timeout 300 --timeout-method thread -k "PRICAI or CLUSSL or foodcom or clussl" > gpurun_out/c3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/c3_tests.log; [ $rc -gt 1 ] && exit $rc
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  env $envs timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline \
    --no-eval > gpurun_out/c3_$tag.json 2> gpurun_out/c3_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/c3_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config3_clussl_foodcom']; print(sys.argv[2], c['dcor'], c['infonce'])" gpurun_out/c3_$tag.json $tag
done
