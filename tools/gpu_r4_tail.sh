#!/bin/bash
# Same-box A/B of the weak board's strip length and tail under the round-4 codegen.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=tools/variants
for rep in 1 2 3; do
  timeout -k 10 400 python tools/ab.py --reps 1 --libs lib,$V/libt025.so,$V/libt075.so,$V/libs768.so,$V/libs1536.so --bench "--workload weak" >> gpurun_out/tail.jsonl 2>> gpurun_out/tail.err || { tail -5 gpurun_out/tail.err; exit 3; }
done
cat gpurun_out/tail.jsonl
