#!/usr/bin/env bash
# One GPU-box session: a kernel trace of the in-tree build (tools/trace_step.sh) then an A/B
# (tools/ab_run.sh) -- both steps under their own time limits, stopping at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-sess}
TAG=$TAG-trace bash tools/trace_step.sh > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
head -3 gpurun_out/$TAG-trace/timeline.txt
TAG=$TAG bash tools/ab_run.sh
