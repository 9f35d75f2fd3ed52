"""Launch latency of small boards (the reference's own image sizes, 16^2 .. 5120^2): median time
of engine.step(turns) per strip height and turns per launch, one JSON line per setting, on the
GPU box.  Small boards are latency-bound: a launch's duration is one wave's serial walk over its
strip + 2k rows, so the strip that fills the GPU with many short walks wins there.

    python tools/small_board.py [--sides 512,4096] [--turns 100]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]


def med_ms(f, n=9):
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
    ap.add_argument("--sides", default="512,4096")
    ap.add_argument("--turns", type=int, default=100)
    ap.add_argument("--strips", default="0,1,2,4,8,16,32,64")
    ap.add_argument("--ks", default="0")
    ap.add_argument("--lib", default="", help="another build of libgolhip.so (same-box A/B)")
    a = ap.parse_args()
    import golhip
    if a.lib:
        from golhip import _lib
        _lib._lib = _lib.load(a.lib, strict=False)
    for side in map(int, a.sides.split(",")):
        ref = None
        for k in map(int, a.ks.split(",")):
            for strip in map(int, a.strips.split(",")):
                try:
                    e = golhip.Engine(side, side, device=0, strip_rows=strip, turns_per_launch=k)
                except golhip.GolError as ex:
                    print(json.dumps({"side": side, "k": k, "strip": strip, "error": str(ex)}), flush=True)
                    continue
                with e:
                    e.load_random(7)
                    ms = med_ms(lambda: e.step(a.turns))
                    e.load_random(7)
                    e.step(a.turns)
                    h = e.hash()
                    info = e.info()
                ref = h if ref is None else ref
                print(json.dumps({"lib": a.lib or "lib", "side": side, "k": info["turns_per_launch"], "layout": info["layout"],
                                  "strip": strip, "strip_used": info.get("strip_rows"), "turns": a.turns,
                                  "ms": ms, "us_per_turn": round(ms * 1e3 / a.turns, 2), "same": h == ref, "hash": h}), flush=True)


if __name__ == "__main__":
    main()
