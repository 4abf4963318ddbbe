#!/usr/bin/env bash
# Round-6 session-4 closing call: same-box A/B of the shipped library against the pre-activation
# build (ab_old/libcgr_mpnn3d.so, commit 701af5c) at cfg2, then the round-end evidence
# (tools/final_session.sh).  Every GPU step has its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_s4final
echo "[s4] $(date +%T) lib A/B cfg2"
bash tools/lib_ab.sh cfg2 ab_old/libcgr_mpnn3d.so gpurun_out/r06_s4final/act_lib_ab_cfg2.txt || exit 1
echo "[s4] $(date +%T) final session"
TAG=r06_s4final CONFIGS="cfg4 cfg5 train_default" bash tools/final_session.sh
