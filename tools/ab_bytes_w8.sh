# Same-box A/B: byte pipe at 6 (default) vs 8 waves per SIMD (byte16k).
set -o pipefail
mkdir -p gpurun_out
GOLHIP_LIB=$PWD/build_exp/libbw8.so timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -k "byte" -x -q --timeout 120 --timeout-method thread > gpurun_out/w8_tests.log 2>&1 || exit 5
for rep in 1 2; do for L in bdef bw8; do for st in 0 145 193; do
  echo -n "$L strip=$st " >> gpurun_out/ab_w8.log
  GOLHIP_LIB=$PWD/build_exp/lib$L.so timeout -k 10 60 python bench.py --workload byte16k --no-cpu-baseline --strip $st --steps 200 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> gpurun_out/ab_w8.log || exit 6
done; done; done
