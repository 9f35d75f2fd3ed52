#!/bin/bash
# The GPU suite with one-round launches up to 16 rounds; the N = 2 share's step plan (rccl1 =
# the N-GPU kernel path) against the 4-round library; row- vs block-grain flags on long ranges.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r4e.log 2>&1 || { tail -30 gpurun_out/pytest_r4e.log; exit 4; }
tail -2 gpurun_out/pytest_r4e.log
for lib in "" tools/variants/libr4.so; do
  timeout -k 10 300 python tools/step_cost.py --board strong2 --variants local,rccl1 --reps 2 ${lib:+--lib $lib} >> gpurun_out/ab4_steps.jsonl 2>> gpurun_out/ab4.err || { tail -5 gpurun_out/ab4.err; exit 3; }
done
for rep in 1 2; do
  for b in "--workload strong262k" "--workload weak --rows-per-gpu 131072 --width 262144 --steps 60 --warmup 60"; do
    timeout -k 10 200 python tools/ab.py --reps 1 --libs lib,tools/variants/libnorowf.so --bench "$b" >> gpurun_out/ab4.jsonl 2>> gpurun_out/ab4.err || { tail -5 gpurun_out/ab4.err; exit 3; }
  done
done
cat gpurun_out/ab4_steps.jsonl gpurun_out/ab4.jsonl
