#!/bin/bash
# Separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE): (a) the HealthRec bench step (Adam is
# its dominant kernel), (b) the SpMM alone on the 10M x 1M x 200M graph.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
cd /tmp && export TMPDIR=/tmp
run() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $OUT/${name}_$TAG -o run -- "$@" > $OUT/${name}_$TAG.log 2>&1 || { echo "$name failed"; tail -5 $OUT/${name}_$TAG.log; exit 1; }
}
run pmc_fetch FETCH_SIZE python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmm-10m
run pmc_write WRITE_SIZE python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmm-10m
run pmc10_fetch FETCH_SIZE python3 $R/tools/bench_spmm.py --chunk 1024 --iters 3
run pmc10_write WRITE_SIZE python3 $R/tools/bench_spmm.py --chunk 1024 --iters 3
python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG adam_kernel spmm_units_kernel | tee $OUT/pmc_$TAG.txt
python3 $R/tools/pmc_traffic.py $OUT/pmc10_fetch_$TAG $OUT/pmc10_write_$TAG spmm_units_kernel | tee -a $OUT/pmc_$TAG.txt
