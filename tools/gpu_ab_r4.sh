#!/bin/bash
# Same-box A/B of library builds on the default bench workloads (tools/ab.py), one JSON line per run.
#   tools/gpu_ab_r4.sh "LIBS" "WORKLOADS" REPS TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
LIBS=$1; WLS=${2:-weak}; REPS=${3:-2}; TAG=${4:-ab}
for w in $WLS; do
  timeout -k 10 900 python tools/ab.py --reps $REPS --libs "$LIBS" --bench "--workload $w" >> gpurun_out/$TAG.jsonl 2>> gpurun_out/$TAG.err || { tail -5 gpurun_out/$TAG.err; exit 3; }
done
cat gpurun_out/$TAG.jsonl
