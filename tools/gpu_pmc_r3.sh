#!/bin/bash
# Separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over the HealthRec bench step (HEAD's kernels),
# summarised per engine timing region into gpurun_out/pmc_traffic_$TAG.json (tools/pmc_regions.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $OUT/${name}_$TAG -o run -- "$@" > $OUT/${name}_$TAG.log 2>&1 || { echo "$name failed"; tail -5 $OUT/${name}_$TAG.log; exit 1; }
}
run pmc_fetch FETCH_SIZE python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmm-10m --no-config5 --no-config3 --no-config1
run pmc_write WRITE_SIZE python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-spmm-10m --no-config5 --no-config3 --no-config1
python3 $R/tools/pmc_regions.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_traffic_$TAG.json \
  "over bench.py --steps 5 --warmup 2 HealthRec leg (tools/gpu_pmc_r3.sh $TAG)"
