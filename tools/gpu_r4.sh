#!/bin/bash
# Round-4 GPU check: the several-process rank tests first, then the whole GPU suite, smoke and the
# default bench line.  tools/gpu_r4.sh [pytest -k expr for the first step]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
K=${1:-}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ranks.py -m gpu -x -v --timeout 200 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_ranks.log 2>&1 || { tail -60 gpurun_out/pytest_ranks.log; exit 3; }
tail -3 gpurun_out/pytest_ranks.log
[ -n "$ONLY_RANKS" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 4; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 5; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 6; }
cat gpurun_out/bench.json
