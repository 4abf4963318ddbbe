#!/usr/bin/env bash
# GPU box: run a prebuilt lab binary under a time limit, output to gpurun_out/<TAG>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-lab}
mkdir -p "$OUT"
BIN=$1; shift
timeout -k 10 ${LAB_TIMEOUT:-120} "$BIN" "$@" > "$OUT/$(basename $BIN).txt" 2>&1
rc=$?
cat "$OUT/$(basename $BIN).txt"
exit $rc
