#!/bin/bash
# Same-box A/B of the weak board's role placement, poll sleep and store policy under the round-4 codegen.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=tools/variants
for rep in 1 2; do
  for b in "--workload weak" "--workload strong262k"; do timeout -k 10 400 python tools/ab.py --reps 1 --libs lib,$V/libplace0.so,$V/libsleep1.so,$V/libstaux0.so --bench "$b" >> gpurun_out/knobs.jsonl 2>> gpurun_out/knobs.err || { tail -5 gpurun_out/knobs.err; exit 3; }; done
done
cat gpurun_out/knobs.jsonl
