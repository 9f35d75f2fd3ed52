"""Reference alive-count series of bench.py's boards (GPU; writes tests/golden/bench_counts.json).

bench.py checks every alive count its run produces (settle, warmup and timed steps) against these
series and reports the result as `parity` (the driver's 8-GPU weak-scaling run then
proves its board, not just its speed).  Each series comes from ONE GPU stepping the whole torus
with one shard (LOCAL transport, no halo exchange, no RCCL): an N-independent path, itself pinned
to the oracle by the tiled-torus tests (tests/test_gpu_configs.py).  The boards are
`Engine.load_random(1)` tori, as bench.py loads them:

  weak N=1,2,4,8   (2^17 * N) x 2^20, a count every 12 turns (bench.py --workload weak at N ranks)
  strong262k       262144 x 262144, every 12 turns (any N: the same board)
  bit64k           65536 x 65536, every 12 turns
  byte16k          16384 x 16384, every 32 turns (bench.py steps it on the byte board; the series
                   here comes from the bit board's band kernels: two kernel families must agree)
  4096 x 65536     every 12 turns: bench.py --rows-per-gpu 2048 --width 65536 at 2 ranks (tests)

    python tools/make_bench_counts.py [--out tests/golden/bench_counts.json] [--only KEY ...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "gol-distributed-final_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# (key, H, W, every, turns): turns cover bench.py's default runs with margin
BOARDS = [
    ("131072x1048576", 1 << 17, 1 << 20, 12, 3000),
    ("262144x1048576", 1 << 18, 1 << 20, 12, 3000),
    ("524288x1048576", 1 << 19, 1 << 20, 12, 3000),
    ("1048576x1048576", 1 << 20, 1 << 20, 12, 3000),
    ("262144x262144", 262144, 262144, 12, 12000),
    ("65536x65536", 65536, 65536, 12, 26400),
    ("16384x16384", 16384, 16384, 32, 160000),
    ("4096x65536", 4096, 65536, 12, 600),  # the 2-rank --share-gpu tests' board (tests/test_gpu_ranks.py)
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "bench_counts.json"))
    ap.add_argument("--only", nargs="*", default=None)
    a = ap.parse_args()
    import golhip
    import bench
    out = {"seed": 1, "boards": {}}
    if os.path.exists(a.out):
        with open(a.out) as f:
            out = json.load(f)
    for key, H, W, every, turns in BOARDS:
        if a.only and key not in a.only:
            continue
        t0 = time.perf_counter()
        with golhip.Engine(H, W, device=0) as e:
            info, topo = e.info(), e.topology()
            assert topo["shards"] == 1 and topo["transport"] == "local", topo
            e.load_random(1)
            counts = []
            chunk = every * 100
            done = 0
            while done < turns:
                n = min(chunk, turns - done)
                counts += [int(c) for c in e.step_counted(n, every)]
                done += n
                print(f"{key}: turn {done}/{turns} ({time.perf_counter() - t0:.1f} s)", flush=True)
        out["boards"][key] = {"H": H, "W": W, "every": every, "counts": counts,
                              "path": f"one GPU, one shard ({topo['transport']}), layout {info['layout']}, "
                                      f"k {info['turns_per_launch']}"}
        print(json.dumps({"board": key, "points": len(counts), "last": counts[-1],
                          "s": round(time.perf_counter() - t0, 1)}), flush=True)
    out["kernel_src"] = bench.kernel_source_hash()
    out["generator"] = "tools/make_bench_counts.py"
    tmp = a.out + ".tmp"
    with open(tmp, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    os.replace(tmp, a.out)


if __name__ == "__main__":
    main()
