#!/bin/bash
# Data-parallel path checks on one GPU: RCCL/model/row-grad tests, the world-1 DP bench (forced exchange)
# under rocprofv3, and a 2-rank gloo rehearsal of bench.py --gpus 2.  Usage: gpu_dp_quick.sh TAG
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py tests/test_models_gpu.py tests/test_rowgrad_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_rccl.log 2>&1; rc=$?; tail -3 gpurun_out/t_rccl.log; [ $rc -eq 0 ] || exit $rc
FR_BENCH_DP1=1 bash tools/gpu_hr_quick.sh ${1:-dp1} 100 || exit 1
FR_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --no-spmm-10m > gpurun_out/dp2_gloo.json 2> gpurun_out/dp2_gloo.err; echo "dp2 rc=$?"; cut -c1-400 gpurun_out/dp2_gloo.json
