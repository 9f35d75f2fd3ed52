#!/bin/bash
# Round-4 final evidence on one GPU box: the whole GPU suite + smoke, the four workloads' profiles
# (tools/profile_all.sh: trace + PMC passes), the in-kernel clocks, and the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=${1:-r04f}
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 3; }
  tail -2 gpurun_out/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 4; }
  tail -1 gpurun_out/smoke.log
fi
bash tools/profile_all.sh $TAG || exit 5
GOL_TL_LIB=tools/variants/libclock.so bash tools/gpu_clock.sh > /dev/null || exit 6
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 7; }
cat gpurun_out/bench.json
