#!/usr/bin/env bash
# Same-box A/B of environment-variable variants of the in-tree build: alternating bench runs, one
# line per run.  VARIANTS="base: rofirst:CGR_RO_MAIN_FIRST=1" (name:VAR=val,VAR=val; empty = none)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abenv}
mkdir -p "$OUT"
ROUNDS=${ROUNDS:-3}
ARGS=${BENCH_ARGS:---steps 60 --warmup 30 --cpu-baseline 0 --profile-steps 0 --collate-bench 0 --infer-bench 0}
for r in $(seq 1 "$ROUNDS"); do
  for v in ${VARIANTS}; do
    name=${v%%:*}
    envs=$(echo "${v#*:}" | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py $ARGS > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" "$OUT/${name}_$r.json" "$name" "$r"
  done
done
