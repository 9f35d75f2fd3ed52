#!/bin/bash
# 4 ranks of config 4's board sharing the one GPU over the IPC transport, each rank started here
# with its own output files and the IPC join traced; LIB: a library variant (tools/bench_lib.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
LIB=${1:-lib}
TAG=${2:-a}
export GOL_IPC_TIMEOUT_MS=30000 GOL_BENCH_STACKS_AFTER_S=40 GOL_IPC_TRACE=1
port=$((29555 + RANDOM % 1000))
pids=""
for r in 0 1 2 3; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=4 LOCAL_WORLD_SIZE=4 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
    timeout -k 10 90 python3 -u tools/bench_lib.py $LIB --workload strong262k --gpus 4 --share-gpu --no-cpu-baseline --settle-s 0 --steps 3 --warmup 1 \
    > gpurun_out/ipc4${TAG}_r$r.out 2> gpurun_out/ipc4${TAG}_r$r.err &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p; c=$?; echo "pid $p rc=$c"; [ $c -ne 0 ] && rc=$c; done
grep -h '^{' gpurun_out/ipc4${TAG}_r0.out | cut -c1-200
exit $rc
