#!/usr/bin/env bash
# One GPU-box session for a stack of changes: pytest -m gpu on each variant of $MIDS
# (build/variants/<name>) and on the in-tree build, then a same-box A/B base / $MIDS / in-tree,
# then a step trace of the in-tree build.  Every step under its own time limit; the first failure
# ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-ab3}
MIDS=${MIDS-}
mkdir -p "gpurun_out/$TAG"
for lib in $([ "${TEST_MIDS:-1}" = 1 ] && for m in $MIDS; do echo build/variants/$m/libcgr_mpnn3d.so; done) ""; do
  if [ -n "$lib" ]; then export CGR_MPNN3D_LIB=$lib; else unset CGR_MPNN3D_LIB; fi
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "gpurun_out/$TAG/pytest.log" 2>&1
  rc=$?; echo "pytest ${lib:-in-tree} rc=$rc"; tail -2 "gpurun_out/$TAG/pytest.log"
  [ $rc -eq 0 ] || exit 1
done
unset CGR_MPNN3D_LIB
export BENCH_ARGS=${BENCH_ARGS:---steps 60 --warmup 30 --cpu-baseline 0 --profile-steps 0}
TAG=$TAG ROUNDS=${ROUNDS:-3} VARIANTS="base:build/variants/base/libcgr_mpnn3d.so $(for m in $MIDS; do echo -n "$m:build/variants/$m/libcgr_mpnn3d.so "; done)new:" \
  bash tools/ab_bench.sh || exit 1
TAG=$TAG-trace bash tools/trace_step.sh > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
head -3 gpurun_out/$TAG-trace/timeline.txt
