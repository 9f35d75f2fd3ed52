#!/bin/bash
# GPU box: correctness subset, timelines, same-box A/B of the product library against
# tools/variants/lib$BASE.so on the bench workloads.  tools/gpu_ab.sh BASE "workload args;..."
set -o pipefail
BASE=${1:-base}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_shards.py -m gpu -x -q --timeout 300 --timeout-method thread -k "band or shards or bench_size or tiled or config or byte" > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 3; }
tail -1 gpurun_out/pytest_ab.log
if [ -f tools/tl/libtimeline.so ]; then
  for W in bit64k byte16k; do timeout -k 10 120 python tools/timeline.py run $W 2>/dev/null || exit 4; done
fi
IFS=';' read -ra WLS <<< "${2:---workload bit64k --steps 40;--workload byte16k --steps 100;--steps 20;--workload strong262k --steps 20}"
for W in "${WLS[@]}"; do
  echo "== $W"
  timeout -k 10 500 python tools/ab.py --reps 2 --libs tools/variants/lib$BASE.so,lib --bench "$W" || exit 5
done
