"""Numbers for BASELINE.md's results table, measured on the GPU box (run there via gpurun).

CPU: the oracle's literal per-cell port of worker.go:15-70 with the broker's slab split (one
pthread per slab) on configs 1-3 (configs 2-3 truncated to one turn; they take minutes per turn
on the CPU), and the word-parallel oracle (64 cells per uint64, one thread) on the same boards.
GPU: config 1 through the broker mirror (Operations.Run of images/512x512.pgm, 100 turns,
Threads = 4: host copies included, as the RPC would), median of 5.
One JSON line per measurement."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]

import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402


def med(f, n=5):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    golden = os.path.join(ROOT, "tests", "golden")
    _, _, b512 = O.read_pgm(os.path.join(golden, "images", "512x512.pgm"), 512, 512)
    threads = min(16, len(os.sched_getaffinity(0)))
    for t in (1, 4, threads):
        s = med(lambda: O.run(b512, 100, t))
        emit(what="cpu literal port", config=1, threads=t, GCUPS=512 * 512 * 100 / s / 1e9)
    w = O.random_words(1, 0, 512, 8)
    s = med(lambda: O.bits_run(w, 100))
    emit(what="cpu word-parallel oracle", config=1, threads=1, GCUPS=512 * 512 * 100 / s / 1e9)
    for cfg, side in ((2, 16384), (3, 65536)):
        words = O.random_words(1, 0, side, side // 64)
        if side <= 16384:
            board = O.unpack(words)
            s = med(lambda: O.run(board, 1, threads), 1)
            emit(what="cpu literal port", config=cfg, threads=threads, turns=1, GCUPS=side * side / s / 1e9)
            del board
        s = med(lambda: O.bits_run(words, 1), 1)
        emit(what="cpu word-parallel oracle", config=cfg, threads=1, turns=1, GCUPS=side * side / s / 1e9)
    import golhip
    ops = golhip.Operations(device=0)
    req = golhip.Request(World=b512, Turns=100, ImageHeight=512, ImageWidth=512, Threads=4)
    res = ops.Run(req)
    gold = O.read_pgm(os.path.join(golden, "check", "images", "512x512x100.pgm"))[2]
    assert np.array_equal(res.World, gold)
    s = med(lambda: ops.Run(req))
    emit(what="gpu Operations.Run (host copies incl.)", config=1, GCUPS=512 * 512 * 100 / s / 1e9, ms=s * 1e3)
    with golhip.Engine(512, 512, device=0) as e:
        e.load_bytes(b512)
        e.step(100)
        s = med(lambda: e.step(100))
        emit(what="gpu engine step (board resident)", config=1, GCUPS=512 * 512 * 100 / s / 1e9, ms=s * 1e3)


if __name__ == "__main__":
    main()
