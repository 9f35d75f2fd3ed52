#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for st in 192 288 576; do
  timeout -k 10 300 python tools/ab.py --reps 1 --libs tools/variants/libpstats.so --bench "--workload bit64k --strip $st" || exit 5
done
timeout -k 10 300 python tools/ab.py --reps 1 --libs tools/variants/libpstats.so,lib --bench "--workload weak" || exit 5
