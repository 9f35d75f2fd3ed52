#!/bin/bash
# Workgroup timelines of the one-round launch: ghost rows (contiguous) vs wrap rows read from the
# board, with and without a kernel of another grid right before the launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export GOL_TL_LIB=$R/tools/variants/libtl.so  # (tools/tl/ does not travel)
for w in strong2 strong8; do
  for opt in "" "--wrap" "--pre 37" "--wrap --pre 37" "" "--wrap"; do
    timeout -k 10 120 python tools/timeline.py run $w $opt >> gpurun_out/tl_r4.jsonl 2>> gpurun_out/tl_r4.err || { tail -5 gpurun_out/tl_r4.err; exit 3; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/tl_r4.jsonl"):
    d = json.loads(l)
    print(d["workload"], d["wrap"], d["pre"], d["event_ms"], d["span_us"], d["resident_frac"], d["cus_used"], d["waves_per_cu"], d["cu_end_us_pct"], d["start_us_pct"])
PY
# the RCCL halo on the compute stream after SERIAL steps (lib) vs on the comm stream (commx)
for lib in "" tools/variants/libcommx.so; do
  for b in strong8 strong2; do
    timeout -k 10 300 python tools/step_cost.py --board $b --variants local,rccl1 --reps 2 ${lib:+--lib $lib} >> gpurun_out/tl_steps.jsonl 2>> gpurun_out/tl_r4.err || { tail -5 gpurun_out/tl_r4.err; exit 3; }
  done
done
grep -h '"board"' gpurun_out/tl_steps.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r4f.log 2>&1 || { tail -30 gpurun_out/pytest_r4f.log; exit 4; }
tail -2 gpurun_out/pytest_r4f.log
