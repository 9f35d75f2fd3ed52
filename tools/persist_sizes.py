"""Persistent multi-round launch vs one launch per step over band board sizes (measurement only):
TCUPS of step_counted(steps * 12, 12) on a random board, both engines, same process."""
import sys, time
sys.path[:0] = ["gol-distributed-final_amd", "."]
import torch
import golhip
torch.cuda.init()
for H, W, steps in [(8192, 8192, 400), (16384, 16384, 200), (32768, 32768, 100), (16384, 65536, 60), (65536, 65536, 40)]:
    res = {}
    for persist in (True, False):
        e = golhip.Engine(H, W, persist=persist)
        e.load_random(1)
        e.step_counted(12 * 3, 12)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c = e.step_counted(12 * steps, 12)
        dt = time.perf_counter() - t0
        res[persist] = (H * W * 12 * steps / dt / 1e12, int(c[-1]), e.hash())
        e.close()
    assert res[True][1:] == res[False][1:], res
    print(f"{H}x{W}: persistent {res[True][0]:.1f} TCUPS, per-launch {res[False][0]:.1f} TCUPS", flush=True)
