#!/usr/bin/env bash
# the driver's bench command (--steps 20 --warmup 5) beside the builder's default
# (50 / 30) on one box, alternating, each with further diagnostic blocks of the same K steps
# timed right after the official one (per-step HIP events), so a slow first block shows up.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-gap}
mkdir -p "$OUT"
ROUNDS=${ROUNDS:-3}
EXTRA=${EXTRA:---cpu-baseline 0 --collate-bench 0 --infer-bench 0}
for r in $(seq 1 "$ROUNDS"); do
  for v in "drv:--steps 20 --warmup 5 --diag-blocks 10" "def:--steps 50 --warmup 30 --diag-blocks 4"; do
    name=${v%%:*}
    args=${v#*:}
    timeout -k 10 300 python bench.py $args $EXTRA > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" || exit $?
    python - "$OUT/${name}_$r.json" "$name" "$r" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
bl = d.get("diag_blocks") or []
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"],
      "roof_us", (d.get("roofline") or {}).get("avg_launch_us"),
      "blocks", [b["ms_per_step"] for b in bl], "ev", [b["event_ms_per_step"] for b in bl],
      "first/last", [b["event_ms_first_last"] for b in bl[:2]])
EOF
  done
done
