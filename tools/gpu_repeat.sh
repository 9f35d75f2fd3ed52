#!/bin/bash
# Bench lines under different warmup/step counts (clock settling), one summary line each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/rep_$n.json 2> gpurun_out/rep_$n.err || { tail -20 gpurun_out/rep_$n.err; exit 5; }
  python -c "import json; d=json.load(open('gpurun_out/rep_$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['steps'], d['warmup'])"
}
run weak3 --workload weak --warmup 3
run weak20 --workload weak --warmup 20
run weak3b --workload weak --warmup 3
run bit64k --workload bit64k --steps 300 --warmup 100
run byte16k --workload byte16k --steps 600 --warmup 200
run strong --workload strong262k --steps 40 --warmup 20
run strong3 --workload strong262k
