"""Sweep the bit-board step kernel parameters (turns per launch k, cells per lane,
strip rows) on one GPU; interleaved rounds in one process (cdna guide §5.4 rule 24).
Prints one JSON line per variant: median / min kernel ms and GCUPS."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]

import torch  # noqa: E402

from golhip.sharded import ShardedBoard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--H", type=int, default=1 << 17)
ap.add_argument("--W", type=int, default=1 << 20)
ap.add_argument("--variants", default="1:32:0,4:32:0,8:32:0,16:32:0,4:64:0,8:64:0,16:64:0,2:128:0,4:128:0,8:128:0",
                help="comma list of k:cells_per_lane:strip (standard layout) or b:k:cells_per_lane:strip (band)")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

def _parse(v):
    f = v.split(":")
    band = f[0] == "b"
    k, cpl, strip = (int(x) for x in f[band:])
    return (band, k, cpl, strip)


variants = [_parse(v) for v in a.variants.split(",")]
boards = {}
for band in sorted({v[0] for v in variants}):
    boards[band] = ShardedBoard(a.H, a.W, turns_per_launch=16, layout="band" if band else "standard")
    boards[band].load_random(1)
res = {v: [] for v in variants}
for r in range(a.rounds):
    for (band, k, cpl, strip) in variants:
        board = boards[band]
        if band:
            board.kern.band_cells_per_lane = cpl
        else:
            board.kern.cells_per_lane = cpl
        board.kern.strip_rows = strip
        board.kmax = k
        board.step(k)  # warm
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            board.step(k)
        e.record()
        torch.cuda.synchronize()
        res[(band, k, cpl, strip)].append(s.elapsed_time(e) / a.reps)
for (band, k, cpl, strip), ms in res.items():
    ms.sort()
    med = ms[len(ms) // 2]
    gcups = a.H * a.W * k / (med * 1e-3) / 1e9
    print(json.dumps({"layout": "band" if band else "standard", "k": k, "cpl": cpl, "strip": strip, "ms_med": round(med, 3), "ms_min": round(ms[0], 3),
                      "GCUPS": round(gcups, 1), "alg_GBs": round(gcups * 0.25, 1),
                      "min_traffic_GBs": round(2 * a.H * a.W / 8 / (med * 1e-3) / 1e9, 1)}), flush=True)
