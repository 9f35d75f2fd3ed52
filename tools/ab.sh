#!/bin/bash
# A/B of library builds on one GPU box: tools/ab.sh "<sweep variants>" libA.so libB.so ...
# (build the libraries with tools/build_variant.sh.)  Runs tools/sweep.py for every library in turn, twice, so box-to-box clock differences
# cancel out of the comparison.  Output: gpurun_out/ab.log
set -o pipefail
V=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for rep in 1 2; do
  for L in "$@"; do
    echo "== $L rep $rep" >> $R/gpurun_out/ab.log
    GOLHIP_LIB=$R/$L timeout -k 10 150 python $R/tools/sweep.py --rounds 2 --variants "$V" >> $R/gpurun_out/ab.log 2>/dev/null || exit 3
  done
done
