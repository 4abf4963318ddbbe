#!/usr/bin/env bash
# GPU box: rocprofv3 kernel trace of a short graph-replayed bench (no serial pass) -> per-step
# timeline (tools/timeline.py) and step spans.  TAG names gpurun_out/<TAG>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-trace}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python bench.py --steps ${STEPS:-20} --warmup 30 --cpu-baseline 0 --profile-steps 0 \
  --collate-bench 0 --infer-bench 0 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(find "$OUT/prof" -name "run_kernel_trace.csv" | head -1)
python tools/step_spans.py "$T"
python tools/timeline.py "$T" 'k_adam$' 3 > "$OUT/timeline.txt"
cat "$OUT/timeline.txt"
