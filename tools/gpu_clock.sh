#!/bin/bash
# In-kernel shader clock of each workload's step kernel (tools/timeline.py clock; the stamp build
# must be at tools/variants/libclock.so: python tools/timeline.py build -DGOL_EXP_CLOCK)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for w in ${1:-weak strong262k bit64k byte16k}; do
  GOL_TL_LIB=tools/variants/libclock.so timeout -k 10 120 python tools/timeline.py clock $w >> gpurun_out/clock.jsonl 2>> gpurun_out/clock.err || { tail -5 gpurun_out/clock.err; exit 3; }
done
cat gpurun_out/clock.jsonl
