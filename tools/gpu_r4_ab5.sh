#!/bin/bash
# Where the N = 2 share's RCCL path loses to the local one with one-round launches: step plans
# (step_cost), then kernel traces of local and rccl1; the whole board against the 4-round library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/step_cost.py --board strong2 --variants local,rccl1,rccl1-overlap,loopback1 --reps 2 >> gpurun_out/ab5_steps.jsonl 2>> gpurun_out/ab5.err || { tail -5 gpurun_out/ab5.err; exit 3; }
timeout -k 10 300 python tools/step_cost.py --board strong8 --variants local,rccl1,loopback1 --reps 2 >> gpurun_out/ab5_steps.jsonl 2>> gpurun_out/ab5.err || { tail -5 gpurun_out/ab5.err; exit 3; }
for v in local rccl1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s2_$v -o run -- python tools/step_cost.py --board strong2 --variants $v --reps 1 > gpurun_out/prof_s2_$v.log 2>&1 || { tail -5 gpurun_out/prof_s2_$v.log; exit 5; }
done
for rep in 1 2; do
  timeout -k 10 200 python tools/ab.py --reps 1 --libs lib,tools/variants/libr4.so --bench "--workload strong262k" >> gpurun_out/ab5.jsonl 2>> gpurun_out/ab5.err || { tail -5 gpurun_out/ab5.err; exit 3; }
done
cat gpurun_out/ab5_steps.jsonl gpurun_out/ab5.jsonl
