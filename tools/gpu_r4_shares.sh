#!/bin/bash
# Per-rank step costs with settled clocks (tools/step_cost.py) for config 4's shares at N = 2/4/8
# and config 5's per-rank board, then the whole 262144^2 board on one GPU (bench strong262k).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for b in ${BOARDS:-strong8 strong4 strong2 weak}; do
  timeout -k 10 400 python tools/step_cost.py --board $b --reps 3 >> gpurun_out/shares.jsonl 2>> gpurun_out/shares.err || { tail -5 gpurun_out/shares.err; exit 3; }
done
timeout -k 10 300 python bench.py --workload strong262k --no-cpu-baseline >> gpurun_out/shares_whole.jsonl 2>> gpurun_out/shares.err || exit 4
timeout -k 10 300 python bench.py --workload strong262k --no-cpu-baseline >> gpurun_out/shares_whole.jsonl 2>> gpurun_out/shares.err || exit 5
wc -l gpurun_out/shares.jsonl; cat gpurun_out/shares_whole.jsonl | cut -c1-300
