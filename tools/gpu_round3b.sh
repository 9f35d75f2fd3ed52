#!/bin/bash
# GPU suite + bench lines of every workload + persistent-vs-per-launch A/B of this build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 3; }
tail -2 gpurun_out/pytest_gpu.log
for w in weak bit64k strong262k byte16k; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 5; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['config']['alive_final'])"
done
timeout -k 10 300 python tools/persist_sizes.py || exit 4
for w in bit64k weak; do
  timeout -k 10 400 python tools/ab.py --reps 1 --libs lib --bench "--workload $w --persist" || exit 6
done
