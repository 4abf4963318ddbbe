#!/usr/bin/env bash
# Round-5 check on one GPU box: smoke, pytest -m gpu, the default bench (cfg2), the unpaired
# timing; every step under its own time limit, stopping at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "[r05] $(date +%T) $*"; }
st smoke
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
st pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 200 \
  --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.txt"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" "$OUT/pytest_gpu.txt" | head -20; exit 1; }
st "bench cfg2 (defaults)"
timeout -k 10 400 python bench.py > "$OUT/bench_cfg2.json" 2> "$OUT/bench_cfg2.err" || { tail -5 "$OUT/bench_cfg2.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_cfg2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
if [ "${UNPAIRED:-1}" = "1" ]; then
  st "unpaired timing"
  timeout -k 10 200 python tools/unpaired_timing.py > "$OUT/unpaired_timing.json" 2> "$OUT/unpaired_timing.err" || { tail -5 "$OUT/unpaired_timing.err"; exit 1; }
  tail -c 600 "$OUT/unpaired_timing.json"
fi
st done
