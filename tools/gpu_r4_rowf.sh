#!/bin/bash
# Same-box A/B of the weak board's role placement, poll sleep and store policy under the round-4 codegen.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=tools/variants
for rep in 1 2 3; do
  for b in "--workload weak"; do timeout -k 10 400 python tools/ab.py --reps 1 --libs lib,$V/liballrowf.so --bench "$b" >> gpurun_out/rowf.jsonl 2>> gpurun_out/rowf.err || { tail -5 gpurun_out/rowf.err; exit 3; }; done
done
cat gpurun_out/rowf.jsonl
