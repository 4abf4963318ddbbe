#!/usr/bin/env bash
# Round-6 GPU check: smoke, the GPU test suite, then optional extra steps ($EXTRA, a command).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06}
mkdir -p "$OUT"
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
tail -15 "$OUT/pytest_gpu.txt"; [ $rc -eq 0 ] || exit 1
if [ -n "${EXTRA:-}" ]; then bash -c "$EXTRA" || exit 1; fi
