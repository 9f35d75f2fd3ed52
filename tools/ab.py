"""Same-box A/B of library builds with bench.py (measurement only).

    python tools/ab.py --reps 2 --libs tools/variants/libA.so,lib --bench "--workload bit64k --steps 30"

Runs bench.py once per (rep, library) in a child process whose golhip binding is pointed at that
library (the product path always loads golhip/libgolhip.so; "lib" = the product library), so
box-to-box clock differences cancel out of the comparison.  One JSON line per run."""
import argparse
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = """
import sys, json
sys.path[:0] = [%r, %r]
import golhip._lib as L
if %r != "lib":
    L._lib = L.load(%r, strict=False)
sys.argv = ["bench.py"] + %r
import bench
bench.main()
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--bench", default="")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    libs = a.libs.split(",")
    for rep in range(a.reps):
        for lib in libs:
            path = lib if lib == "lib" else os.path.join(ROOT, lib)
            code = CHILD % (ROOT, os.path.join(ROOT, "gol-distributed-final_amd"), lib, path,
                            shlex.split(a.bench) + ["--no-cpu-baseline"])
            p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT)
            lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            # (exit 1 with a line: bench.py's parity check failed -- a diagnostic build that computes
            # a wrong board on purpose; its timing is still reported, with the parity verdict)
            if p.returncode != 0 and not (p.returncode == 1 and lines):
                print(json.dumps({"lib": lib, "rep": rep, "error": p.stderr[-800:]}), flush=True)
                sys.exit(3)
            line = json.loads(lines[-1])
            rec = {"bench": a.bench, "lib": lib, "rep": rep, "value": line["value"], "ms_per_step": line["ms_per_step"],
                   "launch_ms": (line["roofline"] or {}).get("launch_ms"),
                   "alive_final": line["config"].get("alive_final"),
                   "parity": (line["config"].get("parity") or {}).get("status")}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
