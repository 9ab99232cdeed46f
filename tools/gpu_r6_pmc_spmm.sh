#!/bin/bash
# Round 6 PMC evidence for the config-4 SpMM: beyond-L2 bytes (FETCH_SIZE, WRITE_SIZE in separate passes)
# of the 10M x 1M Zipf graph (config 4) and of the 10M x 16M uniform-popularity graph (bench.py's
# spmm_dram_uniform) -> gpurun_out/pmc_spmm10m_TAG.json (keys config4, dram_uniform; copy it to profiles/r6/pmc_spmm10m.json).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r6}
mkdir -p $OUT $R/profiles/r6
cd /tmp && export TMPDIR=/tmp
run() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $OUT/${name}_$TAG -o run -- "$@" > $OUT/${name}_$TAG.log 2>&1 \
    || { echo "$name failed"; tail -5 $OUT/${name}_$TAG.log; exit 1; }
}
run c4f FETCH_SIZE python3 $R/tools/spmm10m.py --items 1000000 --seed 0 --iters 2
run c4w WRITE_SIZE python3 $R/tools/spmm10m.py --items 1000000 --seed 0 --iters 2
python3 $R/tools/pmc_spmm10m.py $OUT/c4f_$TAG $OUT/c4w_$TAG $OUT/pmc_spmm10m_$TAG.json config4 "($TAG)" || exit 1
run duf FETCH_SIZE python3 $R/tools/spmm10m.py --items 16000000 --seed 1 --iters 2 --uniform
run duw WRITE_SIZE python3 $R/tools/spmm10m.py --items 16000000 --seed 1 --iters 2 --uniform
python3 $R/tools/pmc_spmm10m.py $OUT/duf_$TAG $OUT/duw_$TAG $OUT/pmc_spmm10m_$TAG.json dram_uniform "($TAG)" || exit 1
cat $OUT/pmc_spmm10m_$TAG.json
timeout -k 10 120 python3 $R/tools/spmm10m.py --items 16000000 --seed 1 --iters 5 --uniform
