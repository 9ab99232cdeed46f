set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "spmm or propagate" > gpurun_out/rev_kt.log 2>&1 || { tail -20 gpurun_out/rev_kt.log; exit 1; }
tail -1 gpurun_out/rev_kt.log
bash tools/gpu_c3_ab.sh rev: fwd:FR_ENGINE_LIB=$R/ab/libfr_engine_fwd.so rev2: fwd2:FR_ENGINE_LIB=$R/ab/libfr_engine_fwd.so
AB_STEPS=300 bash tools/gpu_ab_lib.sh hrev:head hfwd:fwd hrev2:head hfwd2:fwd
