"""One rank of a several-process board (tests/test_gpu_ranks.py starts N of these on the one GPU
of the test box): `python tests/_rank_worker.py '<json>'` builds Engine.rank(..., transport=...)
as rank `rank` of `nranks`, runs one scenario through the C ABI and prints one JSON line.

Scenarios (the parent checks the results against the oracle):
  random     load_random(seed), step_counted(turns, every), hash, alive_count, sha256 of this
             rank's rows (store_words), optionally write_pgm(pgm) (collective)
  pgm        load_pgm(path), step_counted(turns, 1), write_pgm(out), this rank's alive cells
  loadwords  load_random(seed); only rank `writer` overwrites rows [y0, y1) with the given words
             (load_words is not collective); then step_counted(turns, every) and hash
  fault      like random, with `lib` (the spin-fault build) on this rank: the step must fail on
             every rank, then a 1-turn step (no flag waits) must work
  dead       rank `victim` exits after joining; the others' next collective must fail
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gol-distributed-final_amd")]


def main():
    a = json.loads(sys.argv[1])
    import numpy as np

    import golhip
    import golhip._lib as L
    lib = L.load(a["lib"]) if a.get("lib") else None
    uid = bytes.fromhex(a["uid"])
    kw = dict(device=a.get("device", 0), transport=a.get("transport", "ipc"), layout=a.get("layout", "auto"),
              turns_per_launch=a.get("k", 0), step=a.get("step", "auto"))
    if lib is not None:
        kw["library"] = lib
    H, W, n, r = a["H"], a["W"], a["nranks"], a["rank"]
    out = {"rank": r}
    e = golhip.Engine.rank(H, W, n, r, uid, **kw)
    sh = e.shard(0)
    y0, y1 = sh["y0"], sh["y1"]
    out.update(topology=e.topology(), y0=y0, y1=y1, info=e.info())
    sc = a["scenario"]
    if sc == "dead":
        if r == a["victim"]:
            print(json.dumps(out), flush=True)
            os._exit(0)  # joined, then gone: no destroy, no further collective
        try:
            e.load_random(1)
            e.step(24)
            out["error"] = None
        except golhip.GolError as x:
            out["error"] = [x.code, str(x)]
        print(json.dumps(out), flush=True)
        os._exit(0)  # (the engine's collectives cannot complete any more)
    if sc == "fault":
        e.load_random(a["seed"])
        try:
            e.step(a["turns"])
            out["error"] = None
        except golhip.GolError as x:
            out["error"] = [x.code, str(x)]
        e.load_random(a["seed"])
        e.step(1)  # k = 1 has no flag waits: works again on every rank
        out["hash1"] = e.hash()
    elif sc in ("random", "loadwords"):
        e.load_random(a["seed"])
        if sc == "loadwords":
            if r == a["writer"]:
                words = np.array(a["words"], dtype=np.uint64).reshape(-1, W // 64)
                e.load_words(a["wy0"], words)
            out["turn0"] = e.turn
        counts = e.step_counted(a["turns"], a["every"])
        out["counts"] = [int(c) for c in counts]
        out["hash"] = e.hash()
        out["alive"] = e.alive_count()
        out["rows_sha"] = hashlib.sha256(e.store_words(y0, y1).tobytes()).hexdigest()
        if a.get("pgm"):
            e.write_pgm(a["pgm"])
        if a.get("flips"):
            out["flips"] = e.step_flips().tolist()
            out["hash_after_flip"] = e.hash()
    elif sc == "pgm":
        e.load_pgm(a["path"])
        out["counts"] = [int(c) for c in e.step_counted(a["turns"], 1)]
        e.write_pgm(a["out"])
        cells = e.alive_cells()
        out["cells_sha"] = hashlib.sha256(np.ascontiguousarray(cells).tobytes()).hexdigest()
        out["ncells"] = int(len(cells))
    e.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
