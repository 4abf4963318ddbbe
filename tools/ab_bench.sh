#!/usr/bin/env bash
# Same-box A/B of library variants (tools/build_variant.sh): alternating bench runs, one JSON
# value per line.  VARIANTS="base:build/variants/base/libcgr_mpnn3d.so new: tl::--loss,torch"
# (name:lib[:extra bench args, comma-separated]; empty lib = in-tree)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
ROUNDS=${ROUNDS:-3}
ARGS=${BENCH_ARGS:---steps 40 --warmup 5 --cpu-baseline 0 --profile-steps 0}
for r in $(seq 1 "$ROUNDS"); do
  for v in ${VARIANTS}; do
    name=${v%%:*}
    rest=${v#*:}
    lib=${rest%%:*}
    extra=""
    if [ "$rest" != "$lib" ]; then extra=$(echo "${rest#*:}" | tr ',' ' '); fi
    if [ -n "$lib" ]; then export CGR_MPNN3D_LIB=$lib; else unset CGR_MPNN3D_LIB; fi
    timeout -k 10 300 python bench.py $ARGS $extra > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" "$OUT/${name}_$r.json" "$name" "$r"
  done
done
