#!/bin/bash
# Build a library variant for same-box A/B runs: tools/build_variant.sh NAME "-DFLAG=1 ..."
# -> tools/variants/libNAME.so, from a copy of the current sources with its own object dir.
# (The product library has one compiled path; variants exist only as these measurement builds.)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; F=$2
D=$R/tools/variants/src_$N
rm -rf "$D" && mkdir -p "$D"
cp "$R"/gol-distributed-final_amd/csrc/{Makefile,*.cpp,*.h,*.hip} "$D/"
# (environment BANDFLAGS / BYTEFLAGS / KFLAGS, if set, replace the Makefile's scheduler / kernel flags)
make -s -j8 -C "$D" ARCH=gfx950 BUILD=./obj OUT=../lib$N.so INC=$R/include \
    CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -I$R/include -I. $F" \
    ${BANDFLAGS+BANDFLAGS="$BANDFLAGS"} ${BYTEFLAGS+BYTEFLAGS="$BYTEFLAGS"} ${KFLAGS+KFLAGS="$KFLAGS"}
rm -rf "$D"  # (the copied sources are not needed once built)
echo "$R/tools/variants/lib$N.so"
