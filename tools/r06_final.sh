#!/usr/bin/env bash
# Round-6 evidence on one fresh GPU box, every step under its own time limit, stopping at the first
# failure.  PART=1: smoke, pytest -m gpu, the default bench (cfg2, with the CPU baseline), the
# driver's command three times, the 2-rank no-launcher rehearsal.  PART=2: the other bench
# configurations, a rocprofv3 kernel trace + stats of the default bench command, PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06_final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
st() { echo "[final] $(date +%T) $*"; }
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], r.get('kernel'), r.get('avg_launch_us'), r.get('frac'))" "$1"; }
if [ "${PART:-1}" = "1" ]; then
  st smoke
  timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  st pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
  tail -2 "$OUT/pytest_gpu.txt"; [ $rc -eq 0 ] || exit 1
  st "bench cfg2 (defaults)"
  timeout -k 10 400 python bench.py > "$OUT/bench_cfg2.json" 2> "$OUT/bench_cfg2.err" || exit 1
  summ "$OUT/bench_cfg2.json"
  for r in 1 2 3; do
    st "driver command $r"
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_cfg2_driver_$r.json" 2> "$OUT/bench_cfg2_driver_$r.err" || exit 1
    summ "$OUT/bench_cfg2_driver_$r.json"
  done
  st "2 ranks, no launcher (gloo rehearsal on one GPU)"
  env -u WORLD_SIZE -u RANK -u LOCAL_RANK timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 \
    > "$OUT/bench_gloo2_spawned.json" 2> "$OUT/bench_gloo2_spawned.err" || exit 1
  summ "$OUT/bench_gloo2_spawned.json"
else
  for c in ${CONFIGS:-cfg4 cfg5 train_default sweep_b16 sweep_b64 sweep_d5 sweep_max}; do
    st "bench $c"
    timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit 1
    summ "$OUT/bench_$c.json"
  done
  st "rocprofv3 kernel trace of the default bench command"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python bench.py --cpu-baseline 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || exit 1
  st "PMC passes"
  TAG=$TAG bash tools/pmc_profile.sh || exit 1
  st "scatter-add PMC passes"
  TAG=$TAG-scatter bash tools/scatter_pmc.sh > "$OUT/scatter_pmc.log" 2>&1 || exit 1
fi
st done
