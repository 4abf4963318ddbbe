#!/usr/bin/env bash
# Build libcgr_mpnn3d.so variants into build/variants/<name>/ for same-box A/B benchmarking
# (tools/ab_bench.sh):
#   tools/build_variant.sh <rev|WORKTREE> <name> [extra hipcc flags, e.g. -DCGR_REDUCE_MAX_BLOCKS=128]
# then on the GPU box: CGR_MPNN3D_LIB=build/variants/<name>/libcgr_mpnn3d.so python bench.py ...
# The variant's Python side is this checkout's (the C ABI must match).
set -eu
REV=$1
NAME=$2
EXTRA=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$(mktemp -d /tmp/cgr_variant_obj.XXXXXX)
if [ "$REV" = "WORKTREE" ]; then
  SRC=$ROOT
else
  SRC=$(mktemp -d /tmp/cgr_variant.XXXXXX)
  git -C "$ROOT" worktree add --detach "$SRC" "$REV" > /dev/null
  trap 'git -C "$ROOT" worktree remove --force "$SRC"' EXIT
fi
make -C "$SRC/cgr-mpnn-3d_amd/csrc" -j8 OUTDIR="$ROOT/${VARIANT_ROOT:-build/variants}/$NAME" OBJDIR="$OBJ" \
  EXTRA="$EXTRA" > /dev/null
rm -rf "$OBJ"
ls -la "$ROOT/${VARIANT_ROOT:-build/variants}/$NAME/libcgr_mpnn3d.so"
