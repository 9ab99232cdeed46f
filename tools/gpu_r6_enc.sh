#!/bin/bash
# Round 6 encoder evidence: per-phase stamps of workgroup 0 (fused layer micro-benchmark at HealthRec's
# shape), rocprofv3 kernel stats, two SQ counter passes and the FETCH/WRITE bytes of the encoder kernels.
# Usage: tools/gpu_r6_enc.sh TAG [--tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r6a}
mkdir -p $OUT
cd $R
if [ "$2" == "--tests" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_encoder_gpu.py tests/test_dropout_model_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $OUT/enc_tests_$TAG.log 2>&1 || { tail -30 $OUT/enc_tests_$TAG.log; exit 1; }
  tail -1 $OUT/enc_tests_$TAG.log
fi
timeout -k 10 120 python3 $R/tools/bench_encoder.py --phases --no-torch --iters 20 > $OUT/enc_${TAG}_phases.json 2>&1 \
  || { tail -5 $OUT/enc_${TAG}_phases.json; exit 1; }
tail -c 1500 $OUT/enc_${TAG}_phases.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/encprof_${TAG} -o run -- python3 $R/tools/bench_encoder.py \
  --no-torch --iters 30 > $OUT/enc_${TAG}.json 2> $OUT/enc_${TAG}.err || { tail -5 $OUT/enc_${TAG}.err; exit 1; }
f=$(find $OUT/encprof_${TAG} -name "*kernel_stats.csv" | head -1)
grep -E "enc_|Name" "$f" | cut -d, -f1-8
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace -f csv -d $OUT/encpmc_${TAG}_$name -o run -- python3 \
    $R/tools/bench_encoder.py --no-torch --iters 5 > $OUT/encpmc_${TAG}_$name.log 2>&1 \
    || { echo "pass $name failed"; tail -5 $OUT/encpmc_${TAG}_$name.log; return 1; }
  python3 $R/tools/sqpmc_sum.py $(find $OUT/encpmc_${TAG}_$name -name "*counter_collection.csv") "enc_" \
    > $OUT/encpmc_${TAG}_$name.txt && cat $OUT/encpmc_${TAG}_$name.txt
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT || exit 1
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
  SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 1
echo enc evidence done
