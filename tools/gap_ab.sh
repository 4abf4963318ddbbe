#!/usr/bin/env bash
# Round 6: the driver's command with and without the steady-state warmup, alternating (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-gapab}
mkdir -p "$OUT"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for v in "steady:" "nowarm:--min-warmup-ms 0" "def50:--steps 50 --warmup 30"; do
    name=${v%%:*}; args=${v#*:}
    base="--steps 20 --warmup 5"; [ "$name" = def50 ] && base=""
    timeout -k 10 300 python bench.py $base $args --cpu-baseline 0 --collate-bench 0 --infer-bench 0 \
      > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d.get('warmup_steady',{}).get('extra_untimed_steps'), (d.get('roofline') or {}).get('avg_launch_us'))" "$OUT/${name}_$r.json" "$name" "$r"
  done
done
