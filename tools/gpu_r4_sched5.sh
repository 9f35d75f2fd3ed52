#!/bin/bash
# Same-box A/B of scheduling directions per pipeline unit against the product build: band
# (pre-RA top-down / bottom-up; the post-RA machine scheduler bottom-up / top-down), bytes
# (pre-RA top-down / bottom-up).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=tools/variants
for rep in 1 2; do
  for b in "--workload weak" "--workload strong262k"; do
    timeout -k 10 400 python tools/ab.py --reps 1 --libs lib,$V/libb_td.so,$V/libb_bu.so,$V/libb_pbu.so,$V/libb_ptd.so --bench "$b" >> gpurun_out/sched5.jsonl 2>> gpurun_out/sched5.err || { tail -5 gpurun_out/sched5.err; exit 3; }
  done
done
for rep in 1 2 3; do
  timeout -k 10 400 python tools/ab.py --reps 1 --libs lib,$V/liby_td.so,$V/liby_bu.so --bench "--workload byte16k" >> gpurun_out/sched5.jsonl 2>> gpurun_out/sched5.err || { tail -5 gpurun_out/sched5.err; exit 3; }
done
cat gpurun_out/sched5.jsonl
