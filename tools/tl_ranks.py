"""Per-rank / per-wave end times of a timeline .npy (tools/timeline.py run ...): rank = workgroup // cus."""
import sys

import numpy as np

v = np.load(sys.argv[1])
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cus = int(sys.argv[3]) if len(sys.argv) > 3 else 256
t0, t1 = v[:, 0], v[:, 1]
base = t0.min()
s, e = (t0 - base) / 100, (t1 - base) / 100
idx = np.arange(len(v))
wg, wave = idx // P, idx % P
rank = wg // cus
for r in np.unique(rank):
    m = (rank == r) & (wave == P - 1)
    print("rank", r, "n", int(m.sum()), "end us p0/10/50/90/100", [round(float(np.percentile(e[m], q)), 1) for q in (0, 10, 50, 90, 100)])
