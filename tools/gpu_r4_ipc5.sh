#!/bin/bash
# The IPC transport pulling from small send buffers: the several-process GPU tests, then config
# 4's board over 2 and 4 rank processes and the weak board over 2 and 4 on the one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ranks.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_ranks.log 2>&1 || { tail -30 gpurun_out/pytest_ranks.log; exit 3; }
tail -2 gpurun_out/pytest_ranks.log
export GOL_IPC_TIMEOUT_MS=60000
for a in "--workload strong262k --gpus 4" "--workload strong262k --gpus 2" "--workload weak --gpus 2" "--workload weak --gpus 4 --rows-per-gpu 65536"; do
  echo "$a"
  timeout -k 10 240 python3 -u bench.py $a --share-gpu --no-cpu-baseline --steps 10 --warmup 3 >> gpurun_out/share5.jsonl 2>> gpurun_out/share5.err || { tail -5 gpurun_out/share5.err; exit 4; }
done
grep -h '^{' gpurun_out/share5.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); c = d['config']
    print(c['workload'], d['n_gpus'], c['parallelism'], c['transport'], d['value'], d['ms_per_step'], c['alive_final'], c['turns_done'])"
