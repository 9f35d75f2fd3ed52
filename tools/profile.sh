#!/bin/bash
# Profile bench.py's dominant kernel on the GPU box (run from the repo root via gpurun).
#   tools/profile.sh <tag> [bench args...]
# 1) rocprofv3 --kernel-trace --stats of the bench command (kernel durations)
# 2) separate --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ/GRBM activity), one counter block set per pass
# Summarise afterwards (here) with tools/pmc_summary.py <tag> <bench key>.
set -o pipefail
TAG=${1:-r02}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
BENCH="$R/bench.py --no-cpu-baseline $*"
KRE="bits_step|band_step|band_pipe|bytes_step|bytes_blocked|bytes_pipe"
# (the bench's own per-workload steps and warmup: pmc_summary.py averages the steady second half of
# each kernel's dispatches, after the clocks settled)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/bench_trace.log 2>&1 || exit 11
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_BRANCH"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_$N -o run -- python3 $BENCH --steps 3 --warmup 2 > $OUT/pmc_$N.log 2>&1 || exit 12
done
echo done
