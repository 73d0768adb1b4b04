#!/bin/bash
# Build libfhe_gpu_<name>.so from a git ref (committed csrc) for A/B runs.
# usage: tools/lab/build_variant.sh <name> <git-ref> [extra -D flags]
set -eu
NAME=$1; REF=$2; shift 2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REF" node-fhe-accelerate_amd/csrc node-fhe-accelerate_amd/Makefile include | tar -x -C "$TMP"
make -s -C "$TMP/node-fhe-accelerate_amd" -j8 VARIANT=_$NAME EXTRA="-DFHE_NS=fhe_$NAME $*" > /dev/null
cp "$TMP/node-fhe-accelerate_amd/build/libfhe_gpu_$NAME.so" "$ROOT/node-fhe-accelerate_amd/build/"
rm -rf "$TMP"
echo "built build/libfhe_gpu_$NAME.so from $REF"
