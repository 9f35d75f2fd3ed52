#!/bin/bash
# Profile every bench workload (tools/profile.sh) on the GPU box; summarise here afterwards with
#   python tools/pmc_summary.py <tag>_<workload> <bench key>
set -o pipefail
TAG=${1:-r02}
bash tools/profile.sh ${TAG}_weak || exit $?
bash tools/profile.sh ${TAG}_bit64k --workload bit64k || exit $?
bash tools/profile.sh ${TAG}_byte16k --workload byte16k || exit $?
bash tools/profile.sh ${TAG}_strong262k --workload strong262k || exit $?
echo profiled
