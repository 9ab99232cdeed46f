set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in head js4 js16 head js4 js16; do
  if [ $v = head ]; then L=""; else L="FR_ENGINE_LIB=$R/ab/libfr_engine_$v.so"; fi
  env $L timeout -k 10 120 python3 tools/profile_ssl.py 1 > gpurun_out/js_$v.json 2>&1 || { tail -5 gpurun_out/js_$v.json; exit 1; }
  echo "$v $(tail -1 gpurun_out/js_$v.json)"
done
FR_ENGINE_LIB=$R/ab/libfr_engine_js4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "infonce" --timeout 120 --timeout-method thread 2>&1 | tail -1
