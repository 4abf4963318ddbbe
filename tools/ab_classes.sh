#!/usr/bin/env bash
# Same-box A/B of library variants by kernel class: per variant, alternating rounds of
#   bench.py (graph-captured step value) + its instrumented serial pass (per-class device time)
# VARIANTS="base:build/variants/base/libcgr_mpnn3d.so new: noov::CGR_OVERLAP_OPTIM=0"
#   (name:lib[:VAR=v,VAR2=w]; empty lib = in-tree build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abc}
mkdir -p "$OUT"
ROUNDS=${ROUNDS:-2}
CFG=${CFG:-cfg2}
for r in $(seq 1 "$ROUNDS"); do
  for v in ${VARIANTS}; do
    IFS=: read -r name lib envs <<< "$v"
    if [ -n "$lib" ]; then export CGR_MPNN3D_LIB=$lib; else unset CGR_MPNN3D_LIB; fi
    timeout -k 10 300 env ${envs//,/ } python bench.py --config $CFG --steps 40 --warmup 10 --cpu-baseline 0 \
      --collate-bench 0 --infer-bench 0 --profile-steps 10 > "$OUT/${name}_$r.json" \
      2> "$OUT/${name}_$r.err" || { tail -5 "$OUT/${name}_$r.err"; exit 1; }
    python - "$OUT/${name}_$r.json" "$name" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
kb = d["kernel_breakdown"]
top = sorted(kb.items(), key=lambda kv: -kv[1]["ms_per_step"])[:9]
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], " ".join(
    f"{k}:{v['ms_per_step'] * 1e3 / max(v['launches_per_step'], 1):.1f}x{v['launches_per_step']:g}" for k, v in top))
PY
  done
done
