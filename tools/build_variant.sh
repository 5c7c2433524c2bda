#!/bin/bash
# Build libraytracer.so from git revision $1 into ab/$2/ (for tools/ab.py).
set -e
REV=$1; NAME=$2
REPO=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/rt_wt_$NAME
rm -rf "$WT"; git -C "$REPO" worktree prune
git -C "$REPO" worktree add -f "$WT" "$REV" > /dev/null
make -s -C "$WT/rust-swift-raytracer_amd" LIB="$REPO/ab/$NAME" OBJ="/tmp/rt_obj_$NAME" "$REPO/ab/$NAME/libraytracer.so"
git -C "$REPO" worktree remove --force "$WT"
echo "built ab/$NAME/libraytracer.so from $REV"
