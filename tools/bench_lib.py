"""bench.py in this process with the golhip binding pointed at a measurement build of the library
(measurement only; the product path always loads golhip/libgolhip.so):

    python tools/bench_lib.py tools/variants/libX.so [bench.py args...]

One process, no child: safe to run directly under rocprofv3 --pmc."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]

if __name__ == "__main__":
    lib = sys.argv[1]
    import golhip._lib as L
    if lib != "lib":
        L._lib = L.load(os.path.join(ROOT, lib), strict=False)
    sys.argv = ["bench.py"] + sys.argv[2:]
    import bench
    bench.main()
