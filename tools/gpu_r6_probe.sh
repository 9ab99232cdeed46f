echo "nproc $(nproc) cpu_count $(python3 -c 'import os;print(os.cpu_count(), len(os.sched_getaffinity(0)))')"
cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/pids.max 2>/dev/null
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_late_drain_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "infonce or sparse or late or held" > gpurun_out/t_r6b.log 2>&1; tail -5 gpurun_out/t_r6b.log
