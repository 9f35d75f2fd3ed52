#!/bin/bash
# Strip sweep of the persistent multi-round launch (bench.py --strip), one JSON summary line per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
W=${1:-bit64k}; shift  # PERSIST=--persist in the environment: the persistent launch
for st in "$@"; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --strip $st $PERSIST > gpurun_out/sw_${W}_$st.json 2> gpurun_out/sw_${W}_$st.err || { tail -5 gpurun_out/sw_${W}_$st.err; exit 5; }
  python -c "import json; d=json.load(open('gpurun_out/sw_${W}_$st.json')); print('$W', $st, d['value'], d['ms_per_step'], d['config']['alive_final'])"
done
