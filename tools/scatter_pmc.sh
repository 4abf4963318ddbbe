#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE of the standalone scatter-add in both cache states: one counter per
# rocprofv3 run (--pmc + --kernel-trace only), each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-scatter_pmc}
mkdir -p "$OUT"
for state in warm cold; do
  for counter in FETCH_SIZE WRITE_SIZE; do
    lc=$(echo $counter | tr 'A-Z' 'a-z')
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $counter -d "$OUT/pmc_${state}_$lc" -o run \
      --output-format csv -- python tools/scatter_pmc.py run $state > "$OUT/pmc_${state}_$lc.out" \
      2> "$OUT/pmc_${state}_$lc.err" || { echo "pass $state $counter failed"; exit 1; }
    tail -1 "$OUT/pmc_${state}_$lc.out"
  done
done
python tools/scatter_pmc.py collect "$OUT"
