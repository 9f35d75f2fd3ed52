#!/bin/bash
# Pieces (one-round launches of the weak board: each pair slot walks 5 pieces of 7282 rows in turn):
# parity (the GPU suite, with the weak board's exact count at turn 300), then same-box A/B against
# the same source without pieces and against the previous commit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/pytest_pieces_cfg.log 2>&1 || { tail -30 gpurun_out/pytest_pieces_cfg.log; exit 4; }
tail -2 gpurun_out/pytest_pieces_cfg.log
for rep in 1 2 3; do
  timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,tools/variants/libnopieces.so,tools/variants/libhead.so --bench "--workload weak" >> gpurun_out/pieces.jsonl 2>> gpurun_out/pieces.err || { tail -5 gpurun_out/pieces.err; exit 3; }
done
for rep in 1 2; do
  for b in "--workload strong262k" "--workload bit64k" "--workload weak --rows-per-gpu 65536 --width 524288 --steps 40 --warmup 20"; do
    timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,tools/variants/libnopieces.so,tools/variants/libhead.so --bench "$b" >> gpurun_out/pieces.jsonl 2>> gpurun_out/pieces.err || { tail -5 gpurun_out/pieces.err; exit 3; }
  done
done
cat gpurun_out/pieces.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pieces.log 2>&1 || { tail -30 gpurun_out/pytest_pieces.log; exit 5; }
tail -2 gpurun_out/pytest_pieces.log
