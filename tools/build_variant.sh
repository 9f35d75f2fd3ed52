#!/bin/bash
# Build a library variant for same-box A/B runs: tools/build_variant.sh NAME "-DFLAG=1 ..."
# -> build_exp/libNAME.so, from a copy of the current sources with its own object dir.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; F=$2
rm -rf "$R/build_exp/src_$N" && mkdir -p "$R/build_exp/src_$N"
cp "$R"/gol-distributed-final_amd/csrc/{Makefile,*.cpp,*.h,*.hip} "$R/build_exp/src_$N/"
make -s -j8 -C "$R/build_exp/src_$N" ARCH=gfx950 BUILD=./obj OUT=../lib$N.so \
    CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -I$R/include -I. $F"
