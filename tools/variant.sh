#!/bin/bash
# Measurement builds of the library for same-box A/B runs (tools/ab.py, tools/gpu.sh ab) and
# the pipeline kernels' resource usage.  The product library has one compiled path; variants
# exist only as these builds, under tools/variants/ (git-ignored, travels to the GPU box).
#
#   tools/variant.sh flags NAME "-DFLAG=1 ..."  current sources, extra compile flags -> libNAME.so
#                                               (environment BANDFLAGS / BYTEFLAGS / KFLAGS, if set,
#                                               replace the Makefile's scheduler / kernel flags)
#   tools/variant.sh rev REV NAME               every source (and golhip.h) of a git revision
#   tools/variant.sh patch NAME FILE [FLAGS]    current sources with FILE (a patch of csrc/, -p1) applied
#   tools/variant.sh kernels REV NAME           current sources with gol_kernels.hip of REV (the
#                                               kernels of REV behind today's engine and ABI)
#   tools/variant.sh res ["-DFLAG ..."]         VGPRs / LDS / scratch / occupancy of the pipe kernels
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
CS=$R/gol-distributed-final_amd/csrc
V=$R/tools/variants
mkdir -p "$V"

copy_current() {  # dir
  rm -rf "$1" && mkdir -p "$1"
  cp "$CS"/{Makefile,*.cpp,*.h,*.hip} "$1/"
}

case ${1:-} in
  flags)
    N=$2; F=$3; D=$V/src_$N
    copy_current "$D"
    make -s -j8 -C "$D" ARCH=gfx950 BUILD=./obj OUT=../lib$N.so INC=$R/include \
        CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -I$R/include -I. $F" \
        ${BANDFLAGS+BANDFLAGS="$BANDFLAGS"} ${BYTEFLAGS+BYTEFLAGS="$BYTEFLAGS"} ${KFLAGS+KFLAGS="$KFLAGS"}
    rm -rf "$D"
    echo "$V/lib$N.so" ;;
  rev)
    REV=$2; N=$3; D=$V/rev_$N
    rm -rf "$D" && mkdir -p "$D/pkg/csrc" "$D/include"
    for f in $(git -C "$R" ls-tree --name-only "$REV" gol-distributed-final_amd/csrc/); do
      git -C "$R" show "$REV:$f" > "$D/pkg/csrc/$(basename "$f")"
    done
    git -C "$R" show "$REV:include/golhip.h" > "$D/include/golhip.h"
    make -s -j8 -C "$D/pkg/csrc" ARCH=gfx950 BUILD=./obj OUT="$V/lib$N.so" INC="$D/include"
    rm -rf "$D"
    echo "$V/lib$N.so" ;;
  patch)  # current sources with a patch (tools/exp/*.patch, paths relative to csrc/) applied
    N=$2; P=$3; D=$V/src_$N
    copy_current "$D"
    patch -s -d "$D" -p1 < "$R/$P"
    make -s -j8 -C "$D" ARCH=gfx950 BUILD=./obj OUT=../lib$N.so INC=$R/include \
        CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -I$R/include -I. ${4:-}"
    rm -rf "$D"
    echo "$V/lib$N.so" ;;
  kernels)
    REV=$2; N=$3; D=$V/src_$N
    copy_current "$D"
    git -C "$R" show "$REV:gol-distributed-final_amd/csrc/gol_kernels.hip" > "$D/gol_kernels.hip"
    make -s -j8 -C "$D" ARCH=gfx950 BUILD=./obj OUT=../lib$N.so INC=$R/include
    rm -rf "$D"
    echo "$V/lib$N.so" ;;
  res)  # each pipeline in its own translation unit, with the Makefile's scheduler flags
    for tu in band:BANDFLAGS bytes:BYTEFLAGS; do
      sched=$(make -s -C "$CS" -f Makefile -f - print <<< "print: ; @echo \$(${tu#*:})")
      tu=${tu%%:*}
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I"$R/include" -I"$CS" \
        -mllvm -amdgpu-atomic-optimizer-strategy=None $sched ${2:-} --cuda-device-only -c \
        -Rpass-analysis=kernel-resource-usage "$CS/gol_${tu}_pipe.hip" -o /tmp/kres_$tu.o 2>&1 |
        grep -A12 "Function Name: .*pipe_kernel" |
        grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: //'
    done ;;
  *)
    sed -n '2,13p' "$0"; exit 2 ;;
esac
