#!/usr/bin/env bash
# Round-4 GPU session: pytest -m gpu (all, verbose), NT phase stamps (diagnostic variant), the
# default bench, the train.py-default config, and a 2-rank gloo rehearsal of the N>1 bench path.
# Each step under its own limit; a crash / abort / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_s}
mkdir -p "$OUT"
st() { echo "[s] $(date +%T) $*"; }
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 137 ] || [ "$1" -eq 139 ]; }
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  st pytest
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest.log" 2>&1; rc=$?
  tail -4 "$OUT/pytest.log"; grep -E "FAILED|ERROR" "$OUT/pytest.log" | head -20
  fatal $rc && exit 1
fi
if [ -f build/variants/stamps/libcgr_mpnn3d.so ] && [ "${SKIP_STAMPS:-0}" = "0" ]; then
  for mode in 1 0; do
    st "stamps serial=$mode"
    CGR_MPNN3D_LIB=build/variants/stamps/libcgr_mpnn3d.so timeout -k 10 300 \
      python tools/stamp_lab.py --config ${STAMP_CFG:-cfg2} --serial $mode --out "$OUT/stamps_s$mode.json" \
      > "$OUT/stamps_s$mode.txt" 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -5 "$OUT/stamps_s$mode.txt"; exit 1; }
  done
fi
if [ "${SKIP_BENCH:-0}" = "0" ]; then
  st "bench cfg2"
  timeout -k 10 400 python bench.py > "$OUT/bench_cfg2.json" 2> "$OUT/bench_cfg2.err" || { tail -5 "$OUT/bench_cfg2.err"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_cfg2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d.get('inference',{}).get('value'))"
  for c in ${EXTRA_CFGS:-train_default}; do
    st "bench $c"
    timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -5 "$OUT/bench_$c.err"; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  done
fi
if [ "${SKIP_GLOO:-0}" = "0" ]; then
  st "bench 2 ranks gloo (rehearsal of the N>1 path on one GPU)"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo \
    --steps 10 --warmup 3 > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err"; rc=$?
  echo "gloo2 rc=$rc"; tail -c 600 "$OUT/bench_gloo2.json"; fatal $rc && exit 1
fi
st done
if [ "${PROBE:-0}" = "1" ]; then
  st "rccl teardown probe"
  AMD_LOG_LEVEL=${PROBE_LOG:-1} timeout -k 10 240 python -u tools/rccl_teardown_probe.py > "$OUT/probe.log" 2>&1; rc=$?
  echo "probe rc=$rc"; grep -v "^Extension modules" "$OUT/probe.log" | tail -40
fi
if [ -n "${AB_VARIANTS:-}" ]; then
  st "class A/B: $AB_VARIANTS"
  TAG=${TAG:-r04_s}-ab VARIANTS="$AB_VARIANTS" ROUNDS=${AB_ROUNDS:-2} bash tools/ab_classes.sh || exit 1
fi
