#!/bin/bash
# Round 5 PMC + kernel-stats evidence: (1) the config-4 SpMM's beyond-L2 bytes (FETCH_SIZE, WRITE_SIZE in
# separate passes over tools/spmm10m.py: the 1M-item config-4 graph and the 4M-item beyond-MALL graph)
# -> profiles/r5/pmc_spmm10m.json; (2) rocprofv3 --kernel-trace --stats of the HealthRec leg at the
# driver's invocation; (3) the HealthRec leg's per-region PMC bytes -> profiles/r5/pmc_traffic.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r5p}
mkdir -p $OUT $R/profiles/r5
cd /tmp && export TMPDIR=/tmp
run() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $OUT/${name}_$TAG -o run -- "$@" > $OUT/${name}_$TAG.log 2>&1 \
    || { echo "$name failed"; tail -5 $OUT/${name}_$TAG.log; exit 1; }
}
run c4f FETCH_SIZE python3 $R/tools/spmm10m.py --items 1000000 --seed 0 --iters 2
run c4w WRITE_SIZE python3 $R/tools/spmm10m.py --items 1000000 --seed 0 --iters 2
python3 $R/tools/pmc_spmm10m.py $OUT/c4f_$TAG $OUT/c4w_$TAG $R/profiles/r5/pmc_spmm10m.json config4 "($TAG)" || exit 1
run bmf FETCH_SIZE python3 $R/tools/spmm10m.py --items 4000000 --seed 1 --iters 2
run bmw WRITE_SIZE python3 $R/tools/spmm10m.py --items 4000000 --seed 1 --iters 2
python3 $R/tools/pmc_spmm10m.py $OUT/bmf_$TAG $OUT/bmw_$TAG $R/profiles/r5/pmc_spmm10m.json beyond_mall "($TAG)" || exit 1
HR="--no-spmm-10m --no-config3 --no-config5 --no-config1 --no-cpu-baseline --no-eval"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 20 \
  --warmup 5 $HR > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err || { echo rocprof failed; tail -20 $OUT/bench_prof_$TAG.err; exit 1; }
f=$(find $OUT/prof_$TAG -name "*kernel_stats.csv" | head -1); cp "$f" $R/profiles/r5/healthrec_${TAG}_kernel_stats.csv
f=$(find $OUT/prof_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_timeline.py "$f" 12 > $R/profiles/r5/healthrec_step_timeline_${TAG}.txt && tail -3 $R/profiles/r5/healthrec_step_timeline_${TAG}.txt
run pmc_fetch FETCH_SIZE python3 $R/bench.py --steps 5 --warmup 2 $HR
run pmc_write WRITE_SIZE python3 $R/bench.py --steps 5 --warmup 2 $HR
python3 $R/tools/pmc_regions.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $R/profiles/r5/pmc_traffic.json \
  "over bench.py --steps 5 --warmup 2 HealthRec leg (tools/gpu_r5_pmc.sh $TAG)" || exit 1
cp $OUT/bench_prof_$TAG.json $R/profiles/r5/ 2>/dev/null
echo pmc done
