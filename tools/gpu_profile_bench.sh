#!/bin/bash
# GPU box: profiles of every bench workload (tools/profile_all.sh TAG) and one default bench line
# per workload (tools/gpu_bench_all.sh).  Summarise here with tools/pmc_summary.py afterwards.
set -o pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/profile_all.sh $TAG || exit $?
bash tools/gpu_bench_all.sh || exit $?
