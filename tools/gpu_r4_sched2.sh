#!/bin/bash
# Same-box A/B of more machine-scheduler choices: the band translation unit (iterative-ilp,
# iterative-minreg, max-ILP without the post-RA scheduler, max-ILP without memory clustering) and
# the main one for the byte pipeline (max-memory-clause).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
V=tools/variants
for rep in 1 2; do
  for b in "--workload weak" "--workload strong262k" "--workload bit64k"; do
    timeout -k 10 400 python tools/ab.py --reps 1 --libs lib,$V/libitilp.so,$V/libitminreg.so,$V/libnopostra.so,$V/libnocluster.so --bench "$b" >> gpurun_out/sched2.jsonl 2>> gpurun_out/sched2.err || { tail -5 gpurun_out/sched2.err; exit 3; }
  done
done
for rep in 1 2 3; do
  timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,$V/libbmemclause.so --bench "--workload byte16k" >> gpurun_out/sched2.jsonl 2>> gpurun_out/sched2.err || { tail -5 gpurun_out/sched2.err; exit 3; }
done
cat gpurun_out/sched2.jsonl
