#!/bin/bash
# 2-rank rehearsal of the bench's N>1 path on ONE GPU (gloo instead of RCCL: two ranks cannot share a
# device under RCCL).  The 8-GPU run is the driver's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-dpb}
mkdir -p $OUT
cd $R
FR_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 5 --no-cpu-baseline \
  --no-spmm-10m > $OUT/bench_dp2_$TAG.json 2> $OUT/bench_dp2_$TAG.err || { echo dp bench failed; tail -30 $OUT/bench_dp2_$TAG.err; exit 1; }
grep metric $OUT/bench_dp2_$TAG.json | cut -c1-400
