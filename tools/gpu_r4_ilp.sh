#!/bin/bash
# band_pipe_kernel in its own translation unit under the max-ILP scheduler: the GPU suite, a
# same-box A/B against the previous build (libhead), then the final-source profiles (r04g).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 3; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  for b in "--workload weak" "--workload strong262k" "--workload bit64k" "--workload byte16k"; do
    timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,tools/variants/libhead.so --bench "$b" >> gpurun_out/ilp.jsonl 2>> gpurun_out/ilp.err || { tail -5 gpurun_out/ilp.err; exit 4; }
  done
done
cat gpurun_out/ilp.jsonl
SKIP_SUITE=1 bash tools/gpu_r4_final.sh ${1:-r04g}
