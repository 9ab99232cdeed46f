#!/bin/bash
# Round-3 GPU batch: the whole -m gpu suite, the encoder phase profile, the config-4 single vs
# sharded P=1 step under rocprofv3 --stats.  Stops at the first fault/timeout (pytest status 1 =
# failures only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/r3_gate.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|rank [0-9]" $OUT/r3_gate.log | tail -30
[ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u tools/bench_encoder.py --phases > $OUT/enc_bench.json 2>&1 || exit $?
tail -c 1600 $OUT/enc_bench.json
cd /tmp && export TMPDIR=/tmp
for m in single sharded; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c4_$m -o run -- python3 $R/tools/profile_c4.py --mode $m --batch 8192 --steps 3 > $OUT/c4_$m.log 2>&1 || { echo "c4 $m failed"; tail -5 $OUT/c4_$m.log; exit 1; }
  grep ms_per_step $OUT/c4_$m.log; find /tmp/c4_$m -name "*kernel_stats.csv" -exec cp {} $OUT/c4_${m}_kernel_stats.csv \;
done
