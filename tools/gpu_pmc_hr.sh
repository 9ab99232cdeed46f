#!/bin/bash
# Separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over the HealthRec bench step: HBM bytes per
# launch of its kernels (row-gradient Adam, dense Adam, fused encoder, SpMM).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-hr}
cd /tmp && export TMPDIR=/tmp
run() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $OUT/${name}_$TAG -o run -- "$@" > $OUT/${name}_$TAG.log 2>&1 || { echo "$name failed"; tail -5 $OUT/${name}_$TAG.log; exit 1; }
}
run pmc_fetch FETCH_SIZE python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmm-10m --no-config5 --no-config3 --no-config1
run pmc_write WRITE_SIZE python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmm-10m --no-config5 --no-config3 --no-config1
python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG "adam_kernel<true>" "adam_kernel<false>" \
  "adam_lazy_rows_kernel<false>" "adam_lazy_rows_kernel<true>" adam_catch_up_multi_kernel enc_fwd_kernel enc_bwd_kernel spmm_units_kernel | tee $OUT/pmc_$TAG.txt
