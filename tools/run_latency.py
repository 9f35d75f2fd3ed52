"""Where the time of one Operations.Run goes (config 1: images/512x512.pgm, 100 turns), measured
on the GPU box: the whole RPC through the Python mirror, then its pieces through the engine
(board upload, the 100 turns, board download, alive list) and the mirror's list conversion.
Median of 11 after a warm-up call; one JSON line.

    python tools/run_latency.py [--side 512] [--turns 100]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]

import numpy as np  # noqa: E402


def med_ms(f, n=11):
    f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[n // 2] * 1e3, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=512)
    ap.add_argument("--turns", type=int, default=100)
    ap.add_argument("--lib", default="", help="another build of libgolhip.so (same-box A/B)")
    a = ap.parse_args()
    import golhip
    if a.lib:
        from golhip import _lib
        _lib._lib = _lib.load(a.lib, strict=False)
    from golhip.broker import _cells
    H = W = a.side
    path = os.path.join(ROOT, "tests", "golden", "images", f"{a.side}x{a.side}.pgm")
    if os.path.exists(path):
        from oracle import oracle as O
        board = O.read_pgm(path, H, W)[2]
    else:
        rng = np.random.default_rng(1)
        board = (rng.integers(0, 2, (H, W), dtype=np.uint8) * 255)
    ops = golhip.Operations(device=0)
    req = golhip.Request(World=board, Turns=a.turns, ImageHeight=H, ImageWidth=W, Threads=4)
    out = {"what": "Operations.Run latency", "lib": a.lib or "lib", "side": a.side, "turns": a.turns}
    out["run_ms"] = med_ms(lambda: ops.Run(req))
    from golhip._lib import lib
    out["run_no_list_ms"] = med_ms(lambda: ops._call(lib().gol_broker_run, req, alive=False, world=True))
    ops.close()
    with golhip.Engine(H, W, device=0) as e:
        out["load_bytes_ms"] = med_ms(lambda: e.load_bytes(board))
        out[f"step{a.turns}_ms"] = med_ms(lambda: e.step(a.turns))
        out["store_bytes_ms"] = med_ms(lambda: e.store_bytes())
        out["alive_count_ms"] = med_ms(lambda: e.alive_count())
        out["alive_cells_ms"] = med_ms(lambda: e.alive_cells())
        xy = e.alive_cells()
        out["alive_len"] = int(len(xy))
        out["py_cells_ms"] = med_ms(lambda: _cells(xy, len(xy)))  # the Response's CellList
        out["py_list_ms"] = med_ms(lambda: list(_cells(xy, len(xy))), 3)  # materialised as Cells
    out["GCUPS_run"] = round(H * W * a.turns / out["run_ms"] / 1e6, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
