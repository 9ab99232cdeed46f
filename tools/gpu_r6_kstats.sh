#!/bin/bash
# rocprofv3 kernel stats of the HealthRec leg for each library (ab/libfr_engine_NAME.so or "cur"):
#   tools/gpu_r6_kstats.sh TAG NAME...   -> gpurun_out/kstats_TAG_NAME.csv + a per-kernel summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for NAME in "$@"; do
  if [ "$NAME" == "cur" ]; then LIB=""; else LIB=$R/ab/libfr_engine_$NAME.so; fi
  FR_ENGINE_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/ks_${TAG}_$NAME -o run -- python3 \
    $R/bench.py --steps 100 --warmup 10 --no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval \
    > $OUT/ks_${TAG}_$NAME.json 2> $OUT/ks_${TAG}_$NAME.err || { echo "$NAME rocprof failed"; tail -20 $OUT/ks_${TAG}_$NAME.err; exit 1; }
  f=$(find $OUT/ks_${TAG}_$NAME -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kstats_${TAG}_$NAME.csv
  echo "== $NAME"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
    print(f"  {n:48s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.1f} us  tot {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
done
