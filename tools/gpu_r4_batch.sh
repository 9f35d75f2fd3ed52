#!/bin/bash
# Count points reduced in batches (one reduce kernel per run of up to 64 points): the GPU suite,
# then a same-box A/B against the previous build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_batch.log 2>&1 || { tail -40 gpurun_out/pytest_batch.log; exit 3; }
tail -2 gpurun_out/pytest_batch.log
for rep in 1 2 3; do
  for b in "--workload bit64k" "--workload weak" "--workload strong262k"; do
    timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,tools/variants/libprev.so --bench "$b" >> gpurun_out/batch.jsonl 2>> gpurun_out/batch.err || { tail -5 gpurun_out/batch.err; exit 4; }
  done
done
cat gpurun_out/batch.jsonl
