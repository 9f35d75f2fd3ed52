#!/bin/bash
# A/B of the round-4 step changes (wrap rows copied for many-round lone band shards; one-round
# split up to 4 rounds) against the r4 base library, then their parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for rep in 1 2 3; do
  for b in "--workload weak" "--workload strong262k" "--workload bit64k" "--workload weak --rows-per-gpu 65536 --width 262144 --steps 100 --warmup 100"; do
    timeout -k 10 200 python tools/ab.py --reps 1 --libs tools/variants/libr4base.so,lib --bench "$b" >> gpurun_out/ab2.jsonl 2>> gpurun_out/ab2.err || { tail -5 gpurun_out/ab2.err; exit 3; }
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_configs.log 2>&1 || { tail -30 gpurun_out/pytest_configs.log; exit 4; }
tail -2 gpurun_out/pytest_configs.log
cat gpurun_out/ab2.jsonl
