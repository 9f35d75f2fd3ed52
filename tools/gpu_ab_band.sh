#!/bin/bash
# Same-box A/B of band pipeline measurement builds (tools/variants) against the product library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIBS=${LIBS:-lib}
for w in ${WORKLOADS:-weak bit64k}; do
  timeout -k 10 900 python tools/ab.py --reps ${REPS:-2} --libs $LIBS --bench "--workload $w" || exit 5
done
