"""Timing experiment for band-layout k values beyond the library default (e.g. the k = 24
eight-wave pipeline): the board lives in one allocation with KMAX halo rows on both
sides, so any k <= KMAX launches contiguously.  Interleaved rounds in one process;
prints ms per launch, GCUPS and the rate of computed (incl. halo) cell-generations.

    python tools/kexp.py --ks 12,24 [--strips 0,2048]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]

import torch  # noqa: E402

from golhip.sharded import HipKernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--H", type=int, default=1 << 17)
ap.add_argument("--W", type=int, default=1 << 20)
ap.add_argument("--ks", default="12,24")
ap.add_argument("--strips", default="0")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
ks = [int(x) for x in a.ks.split(",")]
strips = [int(x) for x in a.strips.split(",")]
KMAX = max(ks)
H, W = a.H, a.W
Wd = W // 32
kern = HipKernels()
kern.Wd = Wd
st = [torch.zeros((H + 2 * KMAX, Wd), dtype=torch.int32, device="cuda") for _ in range(2)]
mid = [s[KMAX:KMAX + H] for s in st]
kern.random_fill(mid[0], 0, W, 1)
kern.random_fill(mid[1], 0, W, 2)
res = {}
for r in range(a.rounds):
    for k in ks:
        for strip in strips:
            kern.strip_rows = strip
            src, dst = st[0], mid[1]
            args = (src[KMAX - k:KMAX], mid[0], src[KMAX + H:KMAX + H + k], dst, 0, H, k)
            kern.band_step(*args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                kern.band_step(*args)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault((k, strip), []).append(e0.elapsed_time(e1) / a.reps)
for (k, strip), ms in res.items():
    ms.sort()
    med = ms[len(ms) // 2]
    print(json.dumps({"k": k, "strip": strip, "ms_med": round(med, 3), "ms_min": round(ms[0], 3),
                      "GCUPS": round(H * W * k / (med * 1e-3) / 1e9, 1)}), flush=True)
