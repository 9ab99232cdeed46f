#!/bin/bash
# Round 5, batch 3: the whole GPU suite, the SSL replays (mode 1 = normalisation in the lse staging,
# mode 3 = the separate normalize launch), the config-3 leg, then the HealthRec line at the driver's
# invocation and at the default (epoch draws prefetched on a host thread), then A/B specs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${TAG:-b3}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 \
  || { grep -E "FAILED|Error|assert" $OUT/${TAG}_tests.log | head -20; tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
for mode in 1 3 1 3; do
  timeout -k 10 120 python3 tools/profile_ssl.py $mode > $OUT/ssl_${TAG}_m$mode.json 2>&1 || { tail -5 $OUT/ssl_${TAG}_m$mode.json; exit 1; }
  echo "mode $mode: $(tail -1 $OUT/ssl_${TAG}_m$mode.json)"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_ssl_${TAG} -o run -- \
  python3 $R/tools/profile_ssl.py > $OUT/ssl_prof_${TAG}.log 2>&1) || { tail -5 $OUT/ssl_prof_${TAG}.log; exit 1; }
python3 - $(find $OUT/prof_ssl_${TAG} -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if "nce" in n or "dcor" in n:
        print("  ", n[:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
HR="--no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval"
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 $HR > $OUT/${TAG}_hr20_$k.json 2> $OUT/${TAG}_hr20_$k.err \
    || { tail -20 $OUT/${TAG}_hr20_$k.err; exit 1; }
done
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 $HR > $OUT/${TAG}_hr200.json 2> $OUT/${TAG}_hr200.err \
  || { tail -20 $OUT/${TAG}_hr200.err; exit 1; }
for f in $OUT/${TAG}_hr20_*.json $OUT/${TAG}_hr200.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['epoch_sampling']; print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], e['ms_per_epoch'], e['host_draw_ms'], e['steps_ms_per_step'], e['lazy_flush_ms_per_epoch'])" $f
done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-spmm-10m --no-config5 --no-config1 --no-cpu-baseline --no-eval \
  > $OUT/${TAG}_c3.json 2> $OUT/${TAG}_c3.err || { tail -20 $OUT/${TAG}_c3.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config3_clussl_foodcom']; print('c3', c['dcor']['ms_per_step'], c['infonce']['ms_per_step'], c['roofline']['avg_call_ms'], c['roofline']['frac'])" $OUT/${TAG}_c3.json
[ $# -gt 0 ] && AB_STEPS=300 bash tools/gpu_ab_lib.sh "$@"
exit 0
