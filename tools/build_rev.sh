#!/bin/bash
# Build libgolhip.so from the sources of a git revision (same-box A/B against it):
#   tools/build_rev.sh REV NAME  -> tools/variants/libNAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; N=$2
D=$R/tools/variants/rev_$N
rm -rf "$D" && mkdir -p "$D/pkg/csrc" "$D/include"
for f in $(git -C "$R" ls-tree --name-only "$REV" gol-distributed-final_amd/csrc/); do
  git -C "$R" show "$REV:$f" > "$D/pkg/csrc/$(basename $f)"
done
git -C "$R" show "$REV:include/golhip.h" > "$D/include/golhip.h"
make -s -j8 -C "$D/pkg/csrc" ARCH=gfx950 BUILD=./obj OUT=$R/tools/variants/lib$N.so INC="$D/include"
rm -rf "$D"
echo "$R/tools/variants/lib$N.so"
