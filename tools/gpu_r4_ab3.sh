#!/bin/bash
# A/B: one-round split up to 16 rounds (r16) on config 4's whole board and N = 2 share; strip
# lengths 2048 / 4096 (with tail strips) on the weak board; against the product library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for rep in 1 2 3; do
  for b in "--workload strong262k" "--workload weak --rows-per-gpu 131072 --width 262144 --steps 60 --warmup 60"; do
    timeout -k 10 200 python tools/ab.py --reps 1 --libs lib,tools/variants/libr16.so --bench "$b" >> gpurun_out/ab3.jsonl 2>> gpurun_out/ab3.err || { tail -5 gpurun_out/ab3.err; exit 3; }
  done
  timeout -k 10 200 python tools/ab.py --reps 1 --libs lib,tools/variants/libs2048.so,tools/variants/libs4096.so --bench "--workload weak" >> gpurun_out/ab3.jsonl 2>> gpurun_out/ab3.err || { tail -5 gpurun_out/ab3.err; exit 3; }
done
cat gpurun_out/ab3.jsonl
