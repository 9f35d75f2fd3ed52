#!/bin/bash
# Byte pipeline: 2 workgroups per CU (one pair, no lone rank) against 3: speed, then HBM reads
# (FETCH_SIZE) per launch of each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,tools/variants/libbpc2.so --bench "--workload byte16k" >> gpurun_out/bpc.jsonl 2>> gpurun_out/bpc.err || { tail -5 gpurun_out/bpc.err; exit 3; }
done
cat gpurun_out/bpc.jsonl
export TMPDIR=/tmp
for v in lib tools/variants/libbpc2.so; do
  n=$(basename $v .so)
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex bytes_pipe --output-format csv -d $R/gpurun_out/fetch_$n -o run -- python3 $R/tools/bench_lib.py $v --workload byte16k --steps 20 --warmup 5 --settle-s 0 --no-cpu-baseline > $R/gpurun_out/fetch_$n.log 2>&1 || { tail -5 $R/gpurun_out/fetch_$n.log; exit 5; }
done
echo fetch done
