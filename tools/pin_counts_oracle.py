"""Alive-count series of bench.py's boards from the CPU ORACLE (writes tests/golden/oracle_counts.json).

tests/golden/bench_counts.json -- the series every bench line's counts are checked against -- comes
from one GPU stepping the whole torus (tools/make_bench_counts.py).  This script computes the same
series on the CPU with the oracle's word-parallel restatement (oracle/gol_oracle_mt.c: the rule of
gol_oracle.c, multi-threaded and in place), so that
  * tests/test_oracle_counts_cpu.py pins the GPU series to the oracle over every point both hold
    (BASELINE config 2 at 16384^2 and config 3 at 65536^2 for their full 10,000 turns and beyond,
    and the bench's weak and 262144^2 boards over the prefix computed here), and
  * tests/test_gpu_configs.py `test_oracle_count_series` steps each board on the GPU to the
    oracle's last turn and compares every count and the final board's hash.
The boards are `Engine.load_random(1)` tori (oracle.random_words(1, ...)).  Test infrastructure
only: nothing in the product reads the output.

    python tools/pin_counts_oracle.py [--only KEY ...] [--turns N] [--threads T]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# (key, H, W, every, turns): the keys and cadences of tests/golden/bench_counts.json
BOARDS = [
    ("4096x65536", 4096, 65536, 12, 600),
    ("16384x16384", 16384, 16384, 32, 160000),
    ("65536x65536", 65536, 65536, 12, 26400),
    ("131072x1048576", 1 << 17, 1 << 20, 12, 3000),
    ("262144x262144", 262144, 262144, 12, 4800),
    ("262144x1048576", 1 << 18, 1 << 20, 12, 1200),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "oracle_counts.json"))
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--turns", type=int, default=None, help="override the turn count (a multiple of every)")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    import oracle as O

    def save(out):
        tmp = a.out + ".tmp"
        with open(tmp, "w") as f:
            json.dump(out, f, separators=(",", ":"))
        os.replace(tmp, a.out)

    out = {"seed": 1, "boards": {}}
    if os.path.exists(a.out):
        with open(a.out) as f:
            out = json.load(f)
    out["generator"] = "tools/pin_counts_oracle.py (oracle/gol_oracle_mt.c)"
    for key, H, W, every, turns in BOARDS:
        if a.only and key not in a.only:
            continue
        turns = a.turns if a.turns else turns
        assert turns % every == 0
        t0 = time.perf_counter()
        words = O.mt_random_words(1, H, W // 64, a.threads)
        counts: list[int] = []
        # chunks of ~1-2 minutes: progress lines, and the prefix is saved as it grows
        chunk = max(every, (int(3e12 / (H * W)) // every) * every)
        rec = {"H": H, "W": W, "every": every, "turns": 0, "counts": counts, "hash_final": None,
               "path": f"CPU oracle (oracle/gol_oracle_mt.c, {a.threads} threads)"}
        out["boards"][key] = rec
        done = 0
        while done < turns:
            n = min(chunk, turns - done)
            counts += [int(c) for c in O.mt_bits_run(words, n, every, a.threads)]
            done += n
            rec["turns"] = done
            rec["seconds"] = round(time.perf_counter() - t0, 1)
            save(out)
            print(f"{key}: turn {done}/{turns} ({rec['seconds']} s, "
                  f"{H * W * done / (time.perf_counter() - t0) / 1e9:.1f} GCUPS)", flush=True)
        rec["hash_final"] = O.mt_hash_words(words, a.threads)
        rec["seconds"] = round(time.perf_counter() - t0, 1)
        save(out)
        print(json.dumps({"board": key, "turns": done, "points": len(counts), "last": counts[-1],
                          "hash_final": rec["hash_final"], "s": rec["seconds"]}), flush=True)
        del words


if __name__ == "__main__":
    main()
