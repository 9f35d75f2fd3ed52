#!/bin/bash
# The GPU-box runner (run from the repo root through gpurun); every step under its own time limit,
# steps chained so that the first failure ends the call.  Outputs go to gpurun_out/.
#
#   tools/gpu.sh suite [pytest -k expr]     GPU tests (-m gpu) + smoke + the default bench line
#   tools/gpu.sh tests [pytest args...]     GPU tests only (default: the whole -m gpu suite)
#   tools/gpu.sh smoke                      __graft_entry__.smoke()
#   tools/gpu.sh bench [workloads...]       one default bench line per workload (weak bit64k strong262k byte16k)
#   tools/gpu.sh profile TAG [workloads...] per workload: rocprofv3 trace + one --pmc pass per counter set
#                                           (summarise here with tools/pmc_summary.py TAG_<workload> <key>)
#   tools/gpu.sh clock [workloads...]       in-kernel shader clock (needs tools/variants/libclock.so:
#                                           python tools/timeline.py build -DGOL_EXP_CLOCK --out libclock)
#   tools/gpu.sh ab BASE "bench args;..."   same-box A/B of tools/variants/libBASE.so against the product
#   tools/gpu.sh share                      the several-process (IPC) rank tests + --share-gpu bench lines
#   tools/gpu.sh share_parity               the weak board at N = 2 and 4 rank processes on one GPU: parity
#   tools/gpu.sh final TAG                  suite, profile TAG, clock (if built), bench: a round's evidence
#   tools/gpu.sh driver                     the driver's bench command twice + once under rocprofv3 --stats
#                                           (gpurun_out/drv/: bench_1/2.json, bench_trace.json, trace/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
WORKLOADS="weak bit64k strong262k byte16k"
PYT="python -u -m pytest -x --timeout 300 --timeout-method thread"

tests() {
  timeout -k 10 1100 $PYT -q "${@:-tests}" -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 3; }
  tail -2 gpurun_out/pytest_gpu.log
}
smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 4; }
  tail -1 gpurun_out/smoke.log
}
bench_default() {
  timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 5; }
  cat gpurun_out/bench.json
}
bench() {
  for w in ${@:-$WORKLOADS}; do
    timeout -k 10 300 python bench.py --workload $w $BENCH_EXTRA > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 5; }
    python -c "import json; d=json.load(open('gpurun_out/bench_$w.json')); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['launch_ms'], r.get('frac'), d['config']['alive_final'], (d.get('cpu_baseline') or {}).get('value'))"
  done
}
profile_one() {  # tag, bench args...: rocprofv3 --kernel-trace --stats of the bench command, then PMC passes
  local tag=$1; shift
  local out=$R/gpurun_out/prof_$tag
  mkdir -p "$out"
  local bench="$R/bench.py --no-cpu-baseline $*"
  local kre="bits_step|band_step|band_pipe|bytes_step|bytes_blocked|bytes_pipe"
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $bench > $out/bench_trace.log 2>&1) || exit 11
  for P in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_BRANCH"; do
    local n=$(echo $P | cut -d' ' -f1)
    (cd /tmp && export TMPDIR=/tmp &&
     timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$kre" --output-format csv -d $out/pmc_$n -o run -- python3 $bench --steps 3 --warmup 2 > $out/pmc_$n.log 2>&1) || exit 12
  done
  echo "profiled $tag"
}
profile() {
  local tag=$1; shift
  for w in ${@:-$WORKLOADS}; do profile_one ${tag}_$w --workload $w; done
}
clock() {
  for w in ${@:-$WORKLOADS}; do
    GOL_TL_LIB=tools/variants/libclock.so timeout -k 10 120 python tools/timeline.py clock $w >> gpurun_out/clock.jsonl 2>> gpurun_out/clock.err || { tail -5 gpurun_out/clock.err; exit 6; }
  done
  cat gpurun_out/clock.jsonl
}
ab() {
  local base=$1
  IFS=';' read -ra wls <<< "${2:---steps 20;--workload strong262k --steps 20;--workload bit64k --steps 40;--workload byte16k --steps 100}"
  for w in "${wls[@]}"; do
    echo "== $w"
    timeout -k 10 500 python tools/ab.py --reps ${REPS:-2} --libs tools/variants/lib$base.so,lib --bench "$w" || exit 7
  done
}
share() {
  timeout -k 10 600 $PYT -v tests/test_gpu_ranks.py -m gpu > gpurun_out/pytest_ranks.log 2>&1 || { tail -30 gpurun_out/pytest_ranks.log; exit 3; }
  tail -2 gpurun_out/pytest_ranks.log
  export GOL_IPC_TIMEOUT_MS=60000
  for a in "--workload strong262k --gpus 4" "--workload strong262k --gpus 2" "--workload weak --gpus 2" "--workload weak --gpus 4 --rows-per-gpu 65536"; do
    echo "$a"
    timeout -k 10 240 python3 -u bench.py $a --share-gpu --no-cpu-baseline --steps 10 --warmup 3 >> gpurun_out/share.jsonl 2>> gpurun_out/share.err || { tail -5 gpurun_out/share.err; exit 8; }
  done
  tail -4 gpurun_out/share.jsonl
}

share_parity() {  # the weak board as the driver's N = 2 and 4 runs size it, rank processes on this GPU (IPC)
  export GOL_IPC_TIMEOUT_MS=60000
  for n in 2 4; do
    timeout -k 10 300 python3 -u bench.py --gpus $n --share-gpu --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/share_parity_$n.json 2> gpurun_out/share_parity_$n.err || { tail -5 gpurun_out/share_parity_$n.err; exit 8; }
    python3 -c "import json; ls=open('gpurun_out/share_parity_$n.json').read().splitlines(); assert len(ls) == 1, ls; d=json.loads(ls[0]); c=d['config']; print($n, d['value'], c['H'], c['parity']['status'], c['parity']['turns_checked'], c['rank_stats']['exchange_ms'], c['rank_stats']['exchange_wait_ms'])"
  done
}

driver() {  # the round-end driver's own command (bench.py --gpus 1 --steps 20 --warmup 5)
  mkdir -p gpurun_out/drv
  for i in 1 2; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv/bench_$i.json 2> gpurun_out/drv/bench_$i.err || { tail -20 gpurun_out/drv/bench_$i.err; exit 5; }
  done
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/drv/trace -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/drv/bench_trace.json 2> $R/gpurun_out/drv/bench_trace.err) || exit 6
  python3 -c "import json; [print(f, json.load(open('gpurun_out/drv/%s.json' % f))['value']) for f in ('bench_1', 'bench_2', 'bench_trace')]"
}

cmd=${1:-suite}; shift || true
case $cmd in
  suite) tests tests ${1:+-k "$1"} && smoke && bench_default ;;
  tests) tests "$@" ;;
  smoke) smoke ;;
  bench) bench "$@" ;;
  profile) profile "$@" ;;
  clock) clock "$@" ;;
  ab) ab "$@" ;;
  share) share ;;
  share_parity) share_parity ;;
  driver) driver ;;
  final)
    tag=${1:?tag}
    tests tests && smoke && profile $tag && { [ ! -f tools/variants/libclock.so ] || clock; } && bench_default ;;
  *) echo "unknown command $cmd"; exit 2 ;;
esac
