#!/bin/bash
# A frozen copy of an earlier commit's product path (bench.py + recformer_amd/ + include/, its own
# librecformer_hip.so built here) under abtree/<name>, for same-box A/Bs of whole library generations
# against the working tree (tools/gpu/run.sh abtree). abtree/ is git-ignored and travels to the box.
#   bash tools/abtree.sh <name> <commit>
set -e
name=${1:?name}; commit=${2:?commit}
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/abtree/$name
rm -rf "$dst"; mkdir -p "$dst"
git -C "$root" archive "$commit" bench.py recformer_amd include | tar -x -C "$dst"
make -s -C "$dst/recformer_amd/csrc" -j8 >/dev/null
echo "$commit" > "$dst/COMMIT"
ls -la "$dst/recformer_amd/"*.so
