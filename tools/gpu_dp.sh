#!/bin/bash
# Data-parallel checks on one GPU (2 ranks share cuda:0): dp_check (exchanged vs dense gradients,
# graphed vs eager steps) and the 2-rank bench line over gloo.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-dp}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 tests/mp/dp_worker.py > $OUT/dp_check_$TAG.log 2>&1 || { echo dp_check failed; tail -30 $OUT/dp_check_$TAG.log; exit 1; }
grep -E "PASS|FAIL" $OUT/dp_check_$TAG.log | head -5
