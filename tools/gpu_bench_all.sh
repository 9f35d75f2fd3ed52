#!/bin/bash
# One default bench line per workload (the bench's per-workload steps and warmup), summary lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for w in weak bit64k strong262k byte16k; do
  timeout -k 10 300 python bench.py --workload $w $BENCH_EXTRA > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 5; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$w.json')); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['launch_ms'], r.get('frac'), d['config']['alive_final'], (d.get('cpu_baseline') or {}).get('value'))"
done
