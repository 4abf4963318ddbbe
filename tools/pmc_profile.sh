#!/usr/bin/env bash
# PMC counter passes (each its own rocprofv3 run, --pmc + --kernel-trace only) over a short
# eager bench.  Output: gpurun_out/$TAG/pmc_<pass>/...counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
CFG=${CFG:-cfg2}
ARGS="--config $CFG --steps ${STEPS:-3} --warmup 2 --cpu-baseline 0 --graph 0 --profile-steps 0 --min-warmup-ms 0 --collate-bench 0 --infer-bench 0"
run_pass() {
  local name=$1; shift
  echo "[pmc] $(date +%T) pass $name: $*"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/pmc_$name" -o run \
    --output-format csv -- python bench.py $ARGS > "$OUT/pmc_$name.out" 2> "$OUT/pmc_$name.err"
  local rc=$?
  echo "[pmc] pass $name rc=$rc"
  return $rc
}
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
run_pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL || exit $?
run_pass fetch FETCH_SIZE || exit $?
run_pass write WRITE_SIZE || exit $?
run_pass tcc TCC_HIT_sum TCC_MISS_sum || exit $?
echo "[pmc] done"
