#!/bin/bash
# Builds the library of a git revision (default HEAD) as coconut-rust_amd/libcoconut_hip_prev.so, the
# "prev" side of an A/B on one GPU box (tools/gpu_iter.sh, COCONUT_HIP_LIB).  Not shipped; gitignored.
set -euo pipefail
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/coconut_prev_$$
git -C "$R" worktree add -q --detach "$W" "$REV"
trap 'git -C "$R" worktree remove --force "$W"' EXIT
make -C "$W/coconut-rust_amd" -j8 > /dev/null
cp "$W/coconut-rust_amd/libcoconut_hip.so" "$R/coconut-rust_amd/libcoconut_hip_prev.so"
echo "prev = $REV ($(git -C "$R" rev-parse --short "$REV"))"
