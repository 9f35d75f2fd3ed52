set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_shards.py -m gpu -x -q --timeout 300 --timeout-method thread -k "band or shards or bench_size or tiled or config or byte" > gpurun_out/pytest_q4.log 2>&1 || { tail -30 gpurun_out/pytest_q4.log; exit 3; }
tail -2 gpurun_out/pytest_q4.log
timeout -k 10 120 python tools/timeline.py run bit64k > gpurun_out/tl_q4.txt 2>/dev/null || exit 4
timeout -k 10 120 python tools/timeline.py run byte16k >> gpurun_out/tl_q4.txt 2>/dev/null || exit 4
cat gpurun_out/tl_q4.txt
for W in "--workload bit64k --steps 40" "--workload byte16k --steps 100" "--steps 20" "--workload strong262k --steps 20"; do
  echo "== $W"
  timeout -k 10 500 python tools/ab.py --reps 2 --libs tools/variants/libQ1.so,lib --bench "$W" || exit 5
done
