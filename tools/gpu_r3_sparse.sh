#!/bin/bash
# sparse-upstream block plan: kernel tests, config-4 full-size + sharded tests, config-4 step timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_config4_full_gpu.py tests/test_config4_gpu.py tests/test_rccl_gpu.py tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/sparse_tests.log 2>&1
rc=$?; tail -3 $OUT/sparse_tests.log; [ $rc -ne 0 ] && exit $rc
for m in single sharded; do for b in 512 8192; do
  timeout -k 10 300 python tools/profile_c4.py --mode $m --batch $b --steps 3 2>/dev/null | tail -1 || exit 1
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/c4prof_single_sp -o run -- python3 $R/tools/profile_c4.py --mode single --batch 8192 --steps 3 > $OUT/c4_single_sp.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/c4prof_sharded_sp -o run -- python3 $R/tools/profile_c4.py --mode sharded --batch 8192 --steps 3 > $OUT/c4_sharded_sp.log 2>&1 || exit 1
echo ok
