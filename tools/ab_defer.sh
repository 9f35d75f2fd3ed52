set -o pipefail
mkdir -p gpurun_out
GOLHIP_LIB=$PWD/build_exp/libbdefer.so timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -k "byte" -x -q --timeout 120 --timeout-method thread > gpurun_out/defer_tests.log 2>&1 || exit 5
for rep in 1 2 3; do for L in bbase bdefer; do
  echo -n "$L " >> gpurun_out/ab_defer.log
  GOLHIP_LIB=$PWD/build_exp/lib$L.so timeout -k 10 60 python bench.py --workload byte16k --no-cpu-baseline --steps 200 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> gpurun_out/ab_defer.log || exit 6
done; done
