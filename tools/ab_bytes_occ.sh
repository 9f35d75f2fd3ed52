# Same-box A/B of byte-pipe occupancy variants (tools/build_variant.sh builds) on byte16k.
set -o pipefail
mkdir -p gpurun_out
GOLHIP_LIB=$PWD/build_exp/libbwpe6.so timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -k "byte" -x -q --timeout 120 --timeout-method thread > gpurun_out/occ_tests.log 2>&1 || exit 5
for rep in 1 2; do for L in default bwpe6; do for st in 0 193 256; do
  LIB=$PWD/build_exp/lib$L.so; [ $L = default ] && LIB=$PWD/gol-distributed-final_amd/golhip/libgolhip.so
  echo -n "$L strip=$st " >> gpurun_out/ab_occ.log
  GOLHIP_LIB=$LIB timeout -k 10 60 python bench.py --workload byte16k --no-cpu-baseline --strip $st --steps 200 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> gpurun_out/ab_occ.log || exit 6
done; done; done
