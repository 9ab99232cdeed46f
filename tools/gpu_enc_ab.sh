R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encoder_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "encoder or CIKM or HealthRec" > gpurun_out/enc_tests.log 2>&1; rc=$?; tail -2 gpurun_out/enc_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_encoder.py > gpurun_out/encb_new.json 2>/dev/null && tail -c 300 gpurun_out/encb_new.json
FR_ENGINE_LIB=$R/ab/libfr_engine_encH.so timeout -k 10 120 python tools/bench_encoder.py > gpurun_out/encb_old.json 2>/dev/null && tail -c 300 gpurun_out/encb_old.json
AB_STEPS=300 bash tools/gpu_ab_lib.sh n1:head o1:encH n2:head o2:encH
