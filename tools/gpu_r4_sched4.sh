#!/bin/bash
# Same-box A/B of more scheduler choices per pipeline unit against the product build: band
# (no pre-RA scheduling, with / without post-RA; post-RA off alone), bytes (max-memory-clause
# without post-RA, no pre-RA scheduling, post-RA off, both off).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=tools/variants
for rep in 1 2; do
  for b in "--workload weak" "--workload strong262k"; do
    timeout -k 10 400 python tools/ab.py --reps 1 --libs lib,$V/libb_nmnp.so,$V/libb_nm.so,$V/libb_np.so --bench "$b" >> gpurun_out/sched4.jsonl 2>> gpurun_out/sched4.err || { tail -5 gpurun_out/sched4.err; exit 3; }
  done
done
for rep in 1 2 3; do
  timeout -k 10 400 python tools/ab.py --reps 1 --libs lib,$V/liby_mcnp.so,$V/liby_nm.so,$V/liby_np.so,$V/liby_nmnp.so --bench "--workload byte16k" >> gpurun_out/sched4.jsonl 2>> gpurun_out/sched4.err || { tail -5 gpurun_out/sched4.err; exit 3; }
done
cat gpurun_out/sched4.jsonl
