#!/bin/bash
# Both pipeline kernels under their own schedulers (band max-ILP without post-RA, bytes
# max-memory-clause): the GPU suite, a
# same-box A/B against the previous build (libhead), then the final-source profiles (r04i).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 3; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  for b in "--workload weak" "--workload strong262k" "--workload bit64k" "--workload byte16k"; do
    timeout -k 10 300 python tools/ab.py --reps 1 --libs lib,tools/variants/libprev.so --bench "$b" >> gpurun_out/ilp2.jsonl 2>> gpurun_out/ilp2.err || { tail -5 gpurun_out/ilp2.err; exit 4; }
  done
done
cat gpurun_out/ilp2.jsonl
SKIP_SUITE=1 bash tools/gpu_r4_final.sh ${1:-r04i}
