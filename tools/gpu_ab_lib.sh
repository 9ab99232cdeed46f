#!/bin/bash
# HealthRec leg under several engine libraries / env settings:  gpu_ab_lib.sh "tag:LIB:ENV=V ..." ...
# LIB "head" = the in-tree library, else ab/libfr_engine_LIB.so (tools/ab_build.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for spec in "$@"; do
  tag=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; envs=${rest#*:}; [ "$envs" = "$rest" ] && envs=""
  if [ "$lib" = "head" ]; then L=""; else L="FR_ENGINE_LIB=$R/ab/libfr_engine_$lib.so"; fi
  env $L $envs timeout -k 10 300 python bench.py --steps ${AB_STEPS:-50} --warmup 10 --no-spmm-10m --no-config3 --no-config5 \
    --no-config1 --no-cpu-baseline --no-eval > $OUT/ab_$tag.json 2> $OUT/ab_$tag.err || { echo "$tag failed"; tail -5 $OUT/ab_$tag.err; exit 1; }
  python3 - "$OUT/ab_$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
sel = {n: k[n]["avg_ms"] for n in ("encoder_fwd", "encoder_bwd", "spmm_masked", "spmm", "adam_rows_slice") if n in k}
print(sys.argv[2], d["value"], d["ms_per_step"], sel)
PY
done
