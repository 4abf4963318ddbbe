#!/usr/bin/env bash
# PMC passes (one rocprofv3 --pmc run each, kernel-trace only) over a lab binary:
#   TAG=x bash tools/pmc_lab.sh tools/b3_lab [args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmclab}
mkdir -p "$OUT"
BIN=$1; shift
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
    -- "$BIN" $LAB_ARGS > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
LAB_ARGS="$*"
pass sqw SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES || exit 1
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
pass ta TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE || exit 1
pass tcc FETCH_SIZE || exit 1
pass hit TCC_HIT_sum TCC_MISS_sum || exit 1
