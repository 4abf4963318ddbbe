#!/usr/bin/env bash
# Round-6 session-3 GPU step: smoke + GPU tests on the in-tree build, then a same-box A/B over
# $VARIANTS ("name:lib ..."; empty lib = in-tree), alternating, $ROUNDS rounds (cfg2), then one
# instrumented bench of each for the per-kernel serial-pass breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06_s3n}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
  tail -3 "$OUT/pytest_gpu.txt"; [ $rc -eq 0 ] || exit 1
fi
ARGS="--config ${CFG:-cfg2} --steps 100 --warmup 30 --cpu-baseline 0 --collate-bench 0 --infer-bench 0 --profile-steps 0"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for v in $VARIANTS; do
    name=${v%%:*}; lib=${v#*:}
    if [ -n "$lib" ]; then export CGR_MPNN3D_LIB=$PWD/$lib; else unset CGR_MPNN3D_LIB; fi
    timeout -k 10 180 python bench.py $ARGS > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" "$OUT/${name}_$r.json" "$name" "$r"
  done
done
PARGS="--config ${CFG:-cfg2} --steps 50 --warmup 30 --cpu-baseline 0 --collate-bench 0 --infer-bench 0 --profile-steps 10"
for v in $VARIANTS; do
  name=${v%%:*}; lib=${v#*:}
  if [ -n "$lib" ]; then export CGR_MPNN3D_LIB=$PWD/$lib; else unset CGR_MPNN3D_LIB; fi
  timeout -k 10 180 python bench.py $PARGS > "$OUT/${name}_prof.json" 2> "$OUT/${name}_prof.err" || exit 1
done
unset CGR_MPNN3D_LIB
if [ "${TRACE:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv \
    -- python bench.py $PARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit 1
fi
