#!/usr/bin/env bash
# One GPU-box A/B session: pytest -m gpu on the in-tree build, then tools/ab_bench.sh over
# $VARIANTS (default: build/variants/base vs the in-tree library).  TAG names gpurun_out/<TAG>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-ab}
mkdir -p "gpurun_out/$TAG"
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "gpurun_out/$TAG/pytest.log" 2>&1
  rc=$?; tail -3 "gpurun_out/$TAG/pytest.log"; [ $rc -le 1 ] || exit $rc
  [ $rc -eq 0 ] || exit 1
fi
export BENCH_ARGS=${BENCH_ARGS:---steps 60 --warmup 30 --cpu-baseline 0 --profile-steps 0}
TAG=$TAG ROUNDS=${ROUNDS:-3} VARIANTS=${VARIANTS:-"base:build/variants/base/libcgr_mpnn3d.so new:"} \
  bash tools/ab_bench.sh
