mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_wide_gpu.py tests/test_rowgrad_gpu.py tests/test_rccl_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fold_tests.log 2>&1; rc=$?; tail -3 gpurun_out/fold_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_lib.sh fold:head || exit 1
bash tools/gpu_topk_prof.sh a
