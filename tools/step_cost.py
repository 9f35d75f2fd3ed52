"""Per-rank cost of the sharded step structure, measured on one GPU.

    python tools/step_cost.py [--board weak|strong2|strong4|strong8|strong262k|bit64k] [--steps 10]

strongN = the one-GPU share of config 4's 262144^2 board at N ranks (262144/N rows x 262144).
Clocks settle during the first ~0.1-0.2 s of load: every variant first runs
>= --warm-s seconds of steps, and its timed region is >= --timed-s seconds; variants are
interleaved rep by rep.  Each variant steps the same synthetic board (seed 1) with k-turn steps through the
engine (gol_engine_step_counted, counts fused every k turns as bench.py does) and prints one
JSON line: wall ms per step (host clock around the call) and the engine's step timing (HIP
events: first launch of a shard-step to its last).  Variants:
  local         one shard, the engine's choice of step plan (overlap for many-round launches)
  local-overlap one shard, edge rows on the edge stream beside the interior (GOL_STEP_OVERLAP)
  local-edgefirst  edge rows, then the interior, on one stream (GOL_STEP_EDGE_FIRST)
  local-serial  one shard, exchange then one launch (GOL_STEP_SERIAL)
  loopback1     one shard through the LOOPBACK transport (device copies of the plan)
  loopback2     two shards on the same GPU (each half the rows, concurrent)
  rccl1         one shard, RCCL send-to-self (the multi-GPU code path, one rank)
  rccl1-overlap, rccl1-serial   the same with the step plan forced
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]

BOARDS = {"weak": (1 << 17, 1 << 20), "strong2": (131072, 262144), "strong4": (65536, 262144),
          "strong8": (32768, 262144), "bit64k": (65536, 65536), "strong262k": (262144, 262144)}
VARIANTS = {
    "local": dict(),
    "local-overlap": dict(step="overlap"),
    "local-edgefirst": dict(step="edge_first"),
    "local-serial": dict(step="serial"),
    "loopback1": dict(transport="loopback"),
    "loopback2": dict(shards=2, same_device=True, transport="loopback"),
    "rccl1": dict(transport="rccl"),
    "rccl1-overlap": dict(transport="rccl", step="overlap"),
    "rccl1-serial": dict(transport="rccl", step="serial"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--board", default="weak", choices=sorted(BOARDS))
    ap.add_argument("--steps", type=int, default=10, help="timed steps at least")
    ap.add_argument("--warm-s", type=float, default=0.2, help="warmup seconds of steps per variant")
    ap.add_argument("--timed-s", type=float, default=0.15, help="timed seconds at least")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--nocount", action="store_true", help="plain steps (no fused alive count)")
    ap.add_argument("--zero", action="store_true", help="an all-dead board (same instructions, no bit toggling)")
    ap.add_argument("--lib", default="", help="a measurement build of the library (tools/variant.sh)")
    a = ap.parse_args()
    import torch
    import golhip
    if a.lib:
        import golhip._lib as L
        L._lib = L.load(os.path.join(ROOT, a.lib), strict=False)
    torch.cuda.set_device(0)
    H, W = BOARDS[a.board]
    ref = None
    plan = None
    for rep in range(a.reps):
        for name in a.variants.split(","):
            with golhip.Engine(H, W, device=0, **VARIANTS[name]) as e:
                k = e.info()["turns_per_launch"]
                e.load_random(1)
                if a.zero:  # clear shard 0's bits in place (one shard): hipMemset from torch's HIP runtime
                    import ctypes
                    ptr, pitch = e.device_bits()
                    hip = ctypes.CDLL("libamdhip64.so")
                    assert hip.hipMemset(ctypes.c_void_p(ptr), 0, ctypes.c_size_t(H * pitch * 4)) == 0
                    assert hip.hipDeviceSynchronize() == 0
                    assert e.alive_count() == 0
                # warmup and timed steps from the first variant's timing, then the same for all
                # (so every variant ends at the same turn and the results must agree)
                w0, nw = time.perf_counter(), 0
                while (plan is None and (time.perf_counter() - w0 < a.warm_s or nw < 3)) or \
                        (plan is not None and nw < plan[0]):
                    e.step_counted(3 * k, k)
                    nw += 3
                if plan is None:
                    per = (time.perf_counter() - w0) / nw
                    plan = (nw, max(a.steps, int(a.timed_s / per) + 1))
                steps = plan[1]
                e.set_timing(True)
                t0 = time.perf_counter()
                if a.nocount:
                    e.step(steps * k)
                    counts = e.step_counted(0, k)
                else:
                    counts = e.step_counted(steps * k, k)
                dt = time.perf_counter() - t0
                t = e.timing()
                h = e.hash()
            if ref is None:
                ref = (h, counts[-1:].tolist())
            line = {"board": a.board + ("-zero" if a.zero else ""), "variant": name + ("-nocount" if a.nocount else ""), "rep": rep, "k": k,
                    "lib": a.lib or "lib",
                    "warm_steps": nw, "steps": steps,
                    "wall_ms_per_step": round(dt / steps * 1e3, 4), "step_ms": round(t["mean_ms"], 4),
                    "shard_steps": t["launches"], "TCUPS": round(H * W * k * steps / dt / 1e12, 2),
                    "same_result": (h, counts[-1:].tolist()) == ref}
            print(json.dumps(line), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
