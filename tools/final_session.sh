#!/usr/bin/env bash
# Round-end evidence on one fresh GPU box, every step under its own time limit, stopping at the
# first failure: smoke, pytest -m gpu, the default bench (cfg2) and cfg4 / cfg5 lines, a rocprofv3
# kernel trace + stats of the default bench command, then the PMC passes (tools/pmc_profile.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "[final] $(date +%T) $*"; }
st smoke
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
st pytest
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
tail -2 "$OUT/pytest_gpu.txt"; [ $rc -eq 0 ] || exit 1
st "bench cfg2 (defaults)"
timeout -k 10 400 python bench.py > "$OUT/bench_cfg2.json" 2> "$OUT/bench_cfg2.err" || exit 1
python -c "import json; d=json.loads(open('$OUT/bench_cfg2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
for c in ${CONFIGS:-cfg4 cfg5 train_default sweep_b16 sweep_b64}; do
  st "bench $c"
  timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit 1
  python -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'])"
done
if [ "${SKIP_PROF:-0}" = "0" ]; then
  st "rocprofv3 kernel trace of the default bench command"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python bench.py --cpu-baseline 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || exit 1
  st "PMC passes"
  TAG=$TAG bash tools/pmc_profile.sh || exit 1
  st "scatter-add PMC passes"
  TAG=$TAG-scatter bash tools/scatter_pmc.sh > "$OUT/scatter_pmc.log" 2>&1 || exit 1
fi
st done
