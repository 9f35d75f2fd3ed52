#!/bin/bash
# Same-box A/B of the scheduler strategy (max-ilp) against the product build, four workloads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for rep in 1 2; do
  for b in "--workload weak" "--workload strong262k" "--workload bit64k" "--workload byte16k"; do
    timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,tools/variants/libmaxilp.so,tools/variants/libmemclause.so --bench "$b" >> gpurun_out/sched.jsonl 2>> gpurun_out/sched.err || { tail -5 gpurun_out/sched.err; exit 3; }
  done
done
cat gpurun_out/sched.jsonl
# the byte pipeline's polls with s_sleep 1 / 2 between them (SALU per VALU)
for rep in 1 2; do
  timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,tools/variants/libbsleep1.so,tools/variants/libbsleep2.so --bench "--workload byte16k" >> gpurun_out/sched_bytes.jsonl 2>> gpurun_out/sched.err || { tail -5 gpurun_out/sched.err; exit 3; }
done
cat gpurun_out/sched_bytes.jsonl
export TMPDIR=/tmp
for v in lib tools/variants/libbsleep1.so; do
  n=$(basename $v .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --kernel-include-regex bytes_pipe --output-format csv -d gpurun_out/pmc_bytes_$n -o run -- python tools/bench_lib.py $v --workload byte16k --steps 20 --warmup 5 --settle-s 0 --no-cpu-baseline > gpurun_out/pmc_bytes_$n.log 2>&1 || { tail -5 gpurun_out/pmc_bytes_$n.log; exit 5; }
done
echo pmc done
