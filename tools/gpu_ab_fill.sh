#!/bin/bash
# GPU box: band-pipeline parity (engine + config sizes) of the product build, then same-box A/B
# against tools/variants/lib$BASE.so on the band workloads.
set -o pipefail
BASE=${1:-nofill}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_small.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "band or small or config3 or config4 or bench_workload or tiled" > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 3; }
tail -1 gpurun_out/pytest_ab.log
for W in "--workload bit64k" "" "--workload strong262k"; do
  echo "== $W"
  timeout -k 10 500 python tools/ab.py --reps 3 --libs tools/variants/lib$BASE.so,lib --bench "$W" | tee -a gpurun_out/ab_fill.jsonl || exit 5
done
