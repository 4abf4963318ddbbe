#!/usr/bin/env bash
# One GPU-box session: smoke -> pytest -m gpu -> short bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash / timeout (exit >= 2 from pytest, or any
# non-zero from smoke/bench) ends the script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
stage() { echo "[gpu_check] $(date +%T) $*"; }

stage smoke
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
rc=$?; stage "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
[ $rc -eq 0 ] || exit $rc

stage "pytest -m gpu"
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider \
  --timeout 300 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; stage "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || exit $rc

if [ "${SKIP_BENCH:-0}" = "0" ]; then
  stage bench
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 30 --warmup 5 --cpu-seconds 8} \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; stage "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
  [ $rc -eq 0 ] || exit $rc
fi

if [ "${SKIP_PROF:-0}" = "0" ]; then
  stage "rocprofv3 kernel trace"
  # the bench command itself (graph-captured timed steps + the serial instrumented pass), so the
  # per-kernel averages here can be set against the bench line's roofline entry
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python bench.py --steps 20 --warmup 3 --cpu-baseline 0 ${PROF_ARGS:-} \
    > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
  rc=$?; stage "rocprof rc=$rc"
  find "$OUT/prof" -name "*stats*" | head
fi
stage done
