#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05s2
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/r05s2/pytest_gpu.txt 2>&1; rc=$?
tail -2 gpurun_out/r05s2/pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
TAG=r05_ab1 VARIANTS="base: rofirst:CGR_RO_MAIN_FIRST=1" bash tools/ab_env.sh || exit 1
CGR_RO_MAIN_FIRST=1 TAG=r05_tl2 STEPS=20 bash tools/trace_step.sh > gpurun_out/r05_tl2.log 2>&1 || exit 1
head -45 gpurun_out/r05_tl2/timeline.txt
TAG=r05_scatter bash tools/scatter_pmc.sh > gpurun_out/r05_scatter.log 2>&1 || { tail -5 gpurun_out/r05_scatter.log; exit 1; }
tail -40 gpurun_out/r05_scatter.log
