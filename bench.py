"""Benchmark of the Game-of-Life hot path on MI355X (BASELINE.json metric:
cell-updates/s (GCUPS) and % of the roofline at 1/2/4/8 GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload weak|strong262k|bit64k|byte16k]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts its N ranks itself
(child processes, before anything touches a GPU) and prints rank 0's line.

Workloads (a "step" = one pass of the hot path = one k-turn launch over the whole board, with
its halo exchange and the fused AliveCellsCount):
  weak     (default) bit-packed torus of 2^17 rows x 2^20 columns PER GPU, rows sharded over the
           ranks (one process per GPU, libgolhip's rank engine: RCCL halo exchange of k rows per
           launch over xGMI, overlapped with the interior rows).  SURVEY.md §8(d)'s weak-scaling
           config; N = 8 is BASELINE.json config 5's 2^20 x 2^20 torus.
  strong262k  262144 x 262144 bit-packed torus sharded over the N ranks (config 4; total work
           fixed as N grows, "scaling": "strong").
  bit64k   65536 x 65536 bit-packed torus on one GPU (config 3); replicas for N > 1.
  byte16k  16384 x 16384 byte-per-cell torus (config 2): the engine's byte board (GOL_LAYOUT_BYTES),
           k = 32 turns per launch of the byte pipeline; replicas for N > 1.

Inputs are synthetic (splitmix64 Bernoulli(1/2) cells, generated on the GPU) and resident in
HBM before timing.  Rank 0 prints one JSON line.  (GOL_BENCH_STACKS_AFTER_S=N: every thread's
Python stack to stderr every N seconds, for a run that seems stuck.)
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "gol-distributed-final_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "cell-updates/sec (GCUPS) + % HBM roofline at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_GINST = 256 * 4 * 0.5 * 2.4  # wave64 VALU instructions/s: 1024 SIMDs x 1 per 2 cycles x 2.4 GHz
BITS_BYTES_PER_UPDATE = 0.25  # 1 bit read + 1 bit written per cell per turn
BYTES_BYTES_PER_UPDATE = 2.0  # 1 byte read + 1 byte written
# the kernel sources and the flags they are compiled with (a PMC profile is keyed to their hash)
KERNEL_SRCS = [os.path.join(ROOT, "gol-distributed-final_amd", "csrc", f)
               for f in ("gol_kernels.hip", "gol_band_pipe.hip", "gol_bytes_pipe.hip", "Makefile")]
# reference alive-count series of the bench boards (tools/make_bench_counts.py: one GPU, one shard,
# no exchange); every count of a run is checked against them (`parity` in the line)
COUNTS_FIXTURE = os.path.join(ROOT, "tests", "golden", "bench_counts.json")
# the same series from the CPU oracle, over a prefix (tools/pin_counts_oracle.py)
ORACLE_COUNTS = os.path.join(ROOT, "tests", "golden", "oracle_counts.json")
# nominal rates of the settle steps (bench.py --settle-s): ~the measured 1-GPU rates
SETTLE_RATE_BITS = 145e12
SETTLE_RATE_BYTES = 58e12


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default per workload: >= ~0.1 s of GPU work; weak 20)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps first (default per workload: >= ~0.1 s of GPU work, weak 20): the "
                         "GPU's clocks settle during the first ~0.1-0.2 s of load, and 3 steps of the weak "
                         "board (36 ms) left its first timed steps 2.6 %% slower (DESIGN.md §6)")
    ap.add_argument("--workload", default="weak", choices=["weak", "strong262k", "bit64k", "byte16k"])
    ap.add_argument("--k", type=int, default=0,
                    help="turns per launch (temporal blocking); 0 = library default for bit boards "
                         "(12 band / 8 standard), 32 for byte16k")
    ap.add_argument("--strip", type=int, default=0, help="rows per strip (0 = auto)")
    ap.add_argument("--layout", default="auto", choices=["auto", "standard", "band"])
    ap.add_argument("--cpl", type=int, default=0, choices=[0, 32, 64, 128],
                    help="cells per lane of the bit kernels (0 = library default: 128 on the band layout)")
    ap.add_argument("--rows-per-gpu", type=int, default=1 << 17)
    ap.add_argument("--width", type=int, default=1 << 20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--settle-s", type=float, default=0.6,
                    help="before the warmup steps, untimed steps of the same workload for about this many "
                         "seconds of GPU work (a fixed count per workload from a nominal rate): the shader clock "
                         "settles during the first ~0.1-0.2 s of load (DESIGN.md §6), and a short --warmup (the "
                         "driver's 5 weak steps = 58 ms) left the first timed steps on a lower clock; reported as "
                         "config.settle_steps (0 = off)")
    ap.add_argument("--snapshot", default="",
                    help="after the timed steps write the board as a P5 file here (every rank its own "
                         "rows, gol_engine_write_pgm: config 5's snapshot); reported, not part of value")
    ap.add_argument("--share-gpu", action="store_true",
                    help="testing on a 1-GPU box: every rank uses cuda:0 and the sharded workloads (weak, "
                         "strong262k) run the same rank engine over the IPC transport (HIP IPC halo pulls, "
                         "host collectives) instead of RCCL, which refuses two ranks on one GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="orchestration only (no GPU): ranks, barriers and the JSON line, value 0")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # tests: this rank exits at once
    ap.add_argument("--library", default="", help=argparse.SUPPRESS)  # tests: another build of libgolhip.so
    a = ap.parse_args(argv)
    # per-workload defaults: each timed region and each warmup >= ~0.1-0.25 s of GPU work
    steps, warm = {"weak": (20, 20), "strong262k": (40, 20), "bit64k": (300, 100), "byte16k": (600, 200)}[a.workload]
    a.steps = steps if a.steps is None else a.steps
    a.warmup = warm if a.warmup is None else a.warmup
    return a


# ------------------------------------------------------------------ launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(args, timeout_s: float = 900.0) -> int:
    """Start the N ranks as child processes (this process never touches the GPU) and print
    rank 0's JSON line.  Every rank is waited for (bounded by timeout_s); when one fails or the
    time is up, the survivors -- blocked in a collective with the dead rank -- are terminated,
    then killed, and the exit status is nonzero."""
    import tempfile
    port = _free_port()
    procs = []
    out0 = tempfile.TemporaryFile()
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL))
    deadline = time.monotonic() + timeout_s
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        failed = [c for c in codes if c not in (None, 0)]
        if failed or all(c == 0 for c in codes) or time.monotonic() > deadline:
            rc = failed[0] if failed else (0 if all(c == 0 for c in codes) else 124)
            break
        time.sleep(0.2)
    if rc:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        end = time.monotonic() + 10
        for p in procs:
            try:
                p.wait(max(0.1, end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    out0.seek(0)
    sys.stdout.write(out0.read().decode(errors="replace"))
    sys.stdout.flush()
    return rc


# ------------------------------------------------------------------ ranks
class Ranks:
    """torch.distributed (gloo, host side) for the barrier, max-over-ranks timing and sharing the
    RCCL unique id; the board's own halo exchange and reductions are RCCL inside libgolhip."""

    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={self.world}")
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            # gloo's C++ side prints "[Gloo] Rank r is connected to ..." on stdout: to stderr, so
            # that rank 0's stdout holds nothing but the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            finally:
                os.dup2(saved, 1)
                os.close(saved)
            assert dist.get_world_size() == args.gpus
            self.dist = dist
        self.dry = args.dry_run
        if not self.dry:
            import torch
            torch.cuda.set_device(self.local)  # barrier()'s synchronize is then this rank's GPU

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()
        if not self.dry:
            import torch
            torch.cuda.synchronize()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t)
        return float(t.item())

    def gather(self, obj) -> list:
        """obj of every rank, in rank order (on every rank)."""
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def share(self, obj):
        if self.dist is None:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


# ------------------------------------------------------------------ measurement helpers
def kernel_source_hash() -> str:
    h = hashlib.sha256()
    for path in KERNEL_SRCS:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def load_pmc(key):
    """PMC counters per launch of this workload's step kernel (tools/pmc_summary.py), only if they
    were measured on the current kernel sources and build flags (sha256 prefix of gol_kernels.hip,
    gol_band_pipe.hip, gol_bytes_pipe.hip and the Makefile): a stale profile is not used."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            e = json.load(f).get(key)
    except (OSError, ValueError):
        return None, "missing"
    if not e:
        return None, "missing"
    if e.get("kernel_src") != kernel_source_hash():
        return None, "stale (profiled on other kernel sources or flags)"
    return e, e.get("profile")


def parity(ranks, board, every, series):
    """Every alive count of this run (settle, warmup and timed steps: after turns every, 2 every,
    ...) against the reference series of the same board (COUNTS_FIXTURE), on every rank; FAIL on
    any rank fails the line.  With N > 1 ranks this is the check that the sharded path (RCCL halo
    exchange over xGMI, or IPC) computed the same torus as one GPU stepping it whole."""
    ref = None
    try:
        with open(COUNTS_FIXTURE) as f:
            ref = json.load(f)["boards"].get(board)
    except (OSError, ValueError, KeyError):
        pass
    series = [int(c) for c in series]
    if not ref or ref.get("every") != every:
        mine = {"status": "unpinned", "reason": f"no reference series for {board} every {every} turns"}
    else:
        want = ref["counts"]
        n = min(len(want), len(series))
        bad = next((i for i in range(n) if series[i] != want[i]), None)
        if bad is not None:
            mine = {"status": "FAIL", "turn": (bad + 1) * every, "got": series[bad], "want": want[bad]}
        else:
            mine = {"status": "ok" if n == len(series) else "partial", "points": n, "turns_checked": n * every,
                    "turns_done": len(series) * every}
    # the run's counts against the CPU oracle's series of the board, over the turns it holds
    try:
        with open(ORACLE_COUNTS) as f:
            orc = json.load(f)["boards"].get(board)
    except (OSError, ValueError, KeyError):
        orc = None
    if orc and orc.get("every") == every:
        m = min(len(orc["counts"]), len(series))
        bad = next((i for i in range(m) if series[i] != orc["counts"][i]), None)
        mine["oracle"] = {"status": "ok" if bad is None else "FAIL", "turns_checked": m * every}
        if bad is not None:
            mine["status"] = "FAIL"
            mine.setdefault("turn", (bad + 1) * every)
    allr = ranks.gather(mine)
    worst = next((r for r in allr if r["status"] == "FAIL"), None) or \
        next((r for r in allr if r["status"] != "ok"), None) or mine
    out = dict(worst)
    out["reference"] = f"tests/golden/bench_counts.json[{board}] (one GPU, one shard, no exchange)"
    if "oracle" in out:
        out["oracle"]["reference"] = f"tests/golden/oracle_counts.json[{board}] (CPU oracle)"
    if ranks.world > 1:
        out["ranks"] = [r["status"] for r in allr]
    return out


def roofline(kind, launch_ms, cell_updates, pmc, pmc_note):
    """The dominant kernel against its binding roof.  With k turns per launch the bit-board step
    is bound by VALU issue: frac = wave64 VALU instructions per launch (PMC
    SQ_INSTS_VALU) / (1024 SIMDs x 0.5 per cycle x 2.4 GHz x the live launch time).  The HBM side
    (PMC bytes per launch / live time vs 8 TB/s) and the SURVEY §8(d) effective-bandwidth figure
    (algorithmic bytes / time) are reported beside it under their own keys."""
    bpu = BITS_BYTES_PER_UPDATE if kind == "bits" else BYTES_BYTES_PER_UPDATE
    sec = launch_ms * 1e-3
    eff = bpu * cell_updates / sec / 1e9
    traffic = pmc.get("bytes_per_launch") if pmc else None
    hbm = {"achieved": round(traffic / sec / 1e9, 1) if traffic else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(traffic / sec / 1e9 / HBM_PEAK_GBS, 4) if traffic else None}
    r = {"launch_ms": round(launch_ms, 4), "cell_updates_per_launch": cell_updates,
         "effective_GBs": round(eff, 1),
         "effective_basis": f"{bpu} B/cell-update (SURVEY.md §8(d)) x {cell_updates:.4g} cell-updates per launch "
                            f"/ {launch_ms:.3f} ms mean launch (HIP events on the launch stream)",
         "traffic": traffic, "hbm": hbm, "pmc": pmc_note}
    valu = pmc.get("valu_insts_per_launch") if pmc else None
    if valu:
        ach = valu / sec / 1e9
        r.update({"bound": "valu", "achieved": round(ach, 1), "peak": VALU_PEAK_GINST,
                  "unit": "G wave64 VALU inst/s", "frac": round(ach / VALU_PEAK_GINST, 4),
                  # the same kernel at the shader clock its profile measured (the chip lowers its
                  # clock under this load: power), and its work per instruction
                  "profile_clock_GHz": pmc.get("clock_GHz"),
                  "profile_clock_source": pmc.get("clock_source"),
                  "frac_at_profile_clock": round(ach / (VALU_PEAK_GINST / 2.4 * pmc["clock_GHz"]), 4)
                  if pmc.get("clock_GHz") else None,
                  "cell_updates_per_valu_lane_op": round(cell_updates / (valu * 64), 3),
                  "note": "VALU issue of the kernel's own instruction stream; since round 5 a band-layout "
                          "generation is 8 logic ops per 32 cells (two output rows share their middle rows' "
                          "sum; 9 in rounds 3-4, 10 before: DESIGN.md §4.1, §4.1b), so the same frac means "
                          "~12 % more cell-updates/s than in round 4"})
    else:  # no PMC profile of this kernel build: only the HBM side can be stated (None without traffic)
        r.update({"bound": "hbm", "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": hbm["frac"]})
    return r


def cpu_baseline(args):
    """The oracle's literal port of worker.go:15-70 with the broker's slab split (one pthread per
    slab, broker.go:135-206) on config 1: images/512x512.pgm, 100 turns, 4 slabs (the reference's
    broker + 4 workers), plus 1 thread and every allowed core.  The Go reference cannot be built
    (no Go toolchain here or on the GPU box)."""
    import numpy as np
    from oracle import oracle as O
    golden = os.path.join(ROOT, "tests", "golden")
    _, _, board = O.read_pgm(os.path.join(golden, "images", "512x512.pgm"), 512, 512)
    want = O.read_pgm(os.path.join(golden, "check", "images", "512x512x100.pgm"))[2]
    allowed = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    allowed = min(allowed, 16)  # the GPU box's CPU share (16 cores per GPU); os.cpu_count() is the whole host
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    res = {}
    for threads in sorted({1, 4, allowed}):
        times = []
        for _ in range(5):
            t0 = time.perf_counter()
            out = O.run(board, 100, threads)
            times.append(time.perf_counter() - t0)
        assert np.array_equal(out, want), "cpu baseline disagrees with check/images/512x512x100.pgm"
        times.sort()
        res[threads] = 512 * 512 * 100 / times[2] / 1e9
    return {"value": round(res[4], 4), "unit": "GCUPS", "cores": 4, "kind": "port",
            "sample": "config 1: images/512x512.pgm, 100 turns, 4 slabs (one pthread per slab = the broker's 4 "
                      "workers), median of 5, result checked against check/images/512x512x100.pgm; literal "
                      "per-cell port of worker.go:15-70 (oracle/gol_oracle.c), the Go reference cannot be built",
            "GCUPS_1_thread": round(res[1], 4), f"GCUPS_{allowed}_threads": round(res[allowed], 4),
            "cpu_count": os.cpu_count(), "cpu_share": allowed, "cpu_model": model}


# ------------------------------------------------------------------ workloads
def run_bits(args, ranks):
    import golhip
    world, rank = ranks.world, ranks.rank
    if args.workload == "weak":
        H, W, sharded = args.rows_per_gpu * world, args.width, True
    elif args.workload == "strong262k":
        H, W, sharded = 262144, 262144, True
    else:
        H, W, sharded = 65536, 65536, False
    kw = dict(device=ranks.local, turns_per_launch=args.k, strip_rows=args.strip, layout=args.layout,
              cells_per_lane=args.cpl)
    if sharded and world > 1:
        # one process per GPU over RCCL; ranks sharing one GPU (testing) over the IPC transport
        transport = "ipc" if args.share_gpu else "rccl"
        uid = ranks.share(golhip.engine.unique_id(transport) if rank == 0 else None)
        e = golhip.Engine.rank(H, W, world, rank, uid, transport=transport, **kw)
        topo = e.topology()
        assert topo["nranks"] == world and topo["transport"] == transport, topo
    else:
        e = golhip.Engine(H, W, **kw)
        topo = e.topology()
    info = e.info()
    k = info["turns_per_launch"]
    e.load_random(1)
    series = []  # every alive count of the run, for the parity check

    def run_n(n):
        series.extend(e.step_counted(n * k, k).tolist())
    settle = settle_steps(args, run_n, float(H // ranks.world if sharded else H) * W * k, SETTLE_RATE_BITS)
    several = sharded and world > 1
    x = {"exchanges": 0, "mean_ms": 0.0, "wait_ms": 0.0, "transfer_ms": 0.0}
    if args.warmup:
        # several ranks: the halo exchanges are timed during the warmup steps (the same work), so
        # that their events stay out of the timed region
        if several:
            e.set_timing(True, exchanges=True)
        run_n(args.warmup)
        if several:
            x = e.exchange_timing()
            e.set_timing(False)
    ranks.barrier()
    e.set_timing(True)
    t0 = time.perf_counter()
    counts = e.step_counted(args.steps * k, k)  # one launch (+ halo exchange + fused count) per step
    dt = time.perf_counter() - t0
    ranks.barrier()
    t = e.timing()
    e.set_timing(False)
    series.extend(counts.tolist())
    per_rank = rank_stats(ranks, dt, t, x, topo)
    dt = ranks.max(dt)
    par = parity(ranks, f"{H}x{W}", k, series)
    alive = int(counts[-1]) if len(counts) else None
    if not sharded and world > 1:
        cells_total = ranks.sum(H * W)  # independent replicas
        alive = int(ranks.sum(alive))
    else:
        cells_total = H * W
    value = cells_total * k * args.steps / dt
    snap = None
    if args.snapshot:
        ranks.barrier()
        s0 = time.perf_counter()
        e.write_pgm(args.snapshot)
        sdt = ranks.max(time.perf_counter() - s0)
        snap = {"path": args.snapshot, "bytes": H * W, "GB_per_s": round(H * W / sdt / 1e9, 3),
                "note": "device unpack + D2H + pwrite of every rank's rows (PCIe and disk inclusive)"}
    layout = {0: "bytes", 1: "standard", 2: "band"}[2 if info["layout"] == "band" else 1]
    key = f"{args.workload}:{args.rows_per_gpu if args.workload == 'weak' else H}x{W}:k{k}:{layout}"
    if info["cells_per_lane"] != 128:
        key += f":cpl{info['cells_per_lane']}"
    pmc, note = load_pmc(key)
    roof = roofline("bits", t["mean_ms"], t["mean_cell_updates"], pmc, note)
    rpg = args.rows_per_gpu
    rows_name = f"2^{rpg.bit_length() - 1}" if rpg & (rpg - 1) == 0 else str(rpg)
    wname = f"2^{W.bit_length() - 1}" if W & (W - 1) == 0 else str(W)
    name = {"weak": f"weak-{rows_name}x{wname}-per-gpu", "strong262k": "strong-262144x262144",
            "bit64k": "bit-65536x65536"}[args.workload]
    cfg = {"workload": name, "H": H, "W": W, "parallelism": (f"rows{world}" if sharded and world > 1 else
                                   (f"replicas{world}" if world > 1 else "1gpu")),
           "transport": topo["transport"], "turns_per_step": k, "layout": layout,
           "cells_per_lane": info["cells_per_lane"], "strip_rows": args.strip or "auto",
           "alive_count_every_step": True, "alive_final": alive, "turns_done": (settle + args.warmup + args.steps) * k,
           "settle_steps": settle, "timed_launches": t["launches"], "parity": par}
    if world > 1:
        cfg["rank_stats"] = per_rank
    if snap:
        cfg["snapshot"] = snap
    e.close()
    dtype = "u32 (bit-packed, 32 cells/word" + (", column-band layout)" if layout == "band" else ")")
    return value, dt, cfg, roof, dtype


def rank_stats(ranks, wall_s, timing, xtiming, topo):
    """What each rank saw, for a run with N > 1 (SCALE's one run must separate compute imbalance
    from exchange cost): the max / min over ranks of the per-step shard time of the timed steps
    (HIP events around the stepping call on the compute stream, edge launches and exchange waits
    included), of the per-exchange time (an event pair around every halo exchange on the stream it
    runs on -- the RCCL send/recv group, or the IPC copies and flag waits -- measured over the
    warmup steps, so that no per-exchange event sits in the timed region), of the wall time, and
    the rank count each rank's engine reports (RCCL / IPC nranks) with its transport."""
    mine = {"launch_ms": timing["mean_ms"], "exchange_ms": xtiming["mean_ms"], "exchanges": xtiming["exchanges"],
            "exchange_wait_ms": xtiming.get("wait_ms", 0.0), "exchange_transfer_ms": xtiming.get("transfer_ms", 0.0),
            "wall_ms": wall_s * 1e3, "nranks": topo["nranks"], "transport": topo["transport"]}
    allr = ranks.gather(mine)

    def mm(key):
        v = [r[key] for r in allr]
        return {"max": round(max(v), 4), "min": round(min(v), 4)}
    return {"launch_ms": mm("launch_ms"), "exchange_ms": mm("exchange_ms"),
            "exchange_wait_ms": mm("exchange_wait_ms"), "exchange_transfer_ms": mm("exchange_transfer_ms"),
            "wall_ms": mm("wall_ms"),
            "exchanges_per_rank": [r["exchanges"] for r in allr], "nranks_seen": [r["nranks"] for r in allr],
            "transports": sorted({r["transport"] for r in allr}),
            "basis": "per rank: launch_ms = mean step time of its shard over the timed steps (HIP events on the compute "
                     "stream), exchange_ms = mean halo exchange over the warmup steps (events on the exchange's "
                     "stream) = exchange_wait_ms (waiting for the ring neighbours to reach the exchange: IPC READY "
                     "polls; RCCL a one-word send/recv with each neighbour issued first while timed) + "
                     "exchange_transfer_ms (the halo rows); max / min over ranks"}


def settle_steps(args, run_n, cell_updates_per_step, nominal_rate):
    """Untimed steps before the warmup for about args.settle_s seconds of GPU work (the shader
    clock's settling time).  The count comes from a nominal rate (cell-updates/s),
    not from a clock, so every run and every rank of a workload runs the same turns (the sharded
    steps are collective, and the final alive count stays reproducible)."""
    if args.settle_s <= 0:
        return 0
    n = max(1, int(args.settle_s * nominal_rate / cell_updates_per_step + 0.5))
    run_n(n)
    return n


def run_bytes(args, ranks):
    """Config 2: 16384 x 16384 byte-per-cell torus, stepped by the engine on its byte board
    (GOL_LAYOUT_BYTES: the board stays one byte per cell in HBM, as the reference's worker holds
    it; each launch runs k = 32 turns of the byte pipeline, 0/255 bytes packed to bits in
    registers, with the alive count fused).  The same cells as the bit workloads' load_random(1)."""
    import golhip
    H = W = 16384
    e = golhip.Engine(H, W, device=ranks.local, turns_per_launch=args.k, strip_rows=args.strip, layout="bytes")
    info = e.info()
    assert info["layout"] == "bytes", info
    k = info["turns_per_launch"]
    e.load_random(1)
    series = []

    def run_n(n):
        series.extend(e.step_counted(n * k, k).tolist())
    settle = settle_steps(args, run_n, float(H) * W * k, SETTLE_RATE_BYTES)
    if args.warmup:
        run_n(args.warmup)
    ranks.barrier()
    e.set_timing(True)
    t0 = time.perf_counter()
    counts = e.step_counted(args.steps * k, k)  # one launch (+ fused count) per step
    dt = time.perf_counter() - t0
    ranks.barrier()
    t = e.timing()
    e.set_timing(False)
    e.close()
    series.extend(counts.tolist())
    par = parity(ranks, f"{H}x{W}", k, series)
    dt = ranks.max(dt)
    value = H * W * ranks.world * k * args.steps / dt
    alive = int(counts[-1]) if len(counts) else None
    if ranks.world > 1:
        alive = int(ranks.sum(alive))  # independent replicas
    pmc, note = load_pmc(f"byte16k:{H}x{W}:k{k}:bytes")
    roof = roofline("bytes", t["mean_ms"], t["mean_cell_updates"], pmc, note)
    cfg = {"workload": "byte-16384x16384", "H": H, "W": W, "turns_per_step": k, "layout": "bytes",
           "parallelism": f"replicas{ranks.world}" if ranks.world > 1 else "1gpu",
           "alive_count_every_step": True, "alive_final": alive, "turns_done": (settle + args.warmup + args.steps) * k,
           "settle_steps": settle, "parity": par}
    return value, dt, cfg, roof, "u8 (byte per cell)"


def main():
    args = parse()
    if os.environ.get("GOL_BENCH_STACKS_AFTER_S"):  # debugging a stuck run: every thread's stack to stderr
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["GOL_BENCH_STACKS_AFTER_S"]), repeat=True)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    if args.k <= 0 and args.workload == "byte16k":
        args.k = 32  # pipelined byte kernel, 8 waves x 4 turns
    if int(os.environ.get("RANK", "0")) == args.fail_rank:
        sys.exit(3)  # (tests/test_bench_cpu.py: the other ranks wait in a collective for it)
    if args.library:  # (tests: a fault-injection build must fail the line's parity check)
        import golhip
        golhip._lib._lib = golhip._lib.load(os.path.abspath(args.library))
    ranks = Ranks(args)
    if args.dry_run:
        ranks.barrier()
        wall = 0.001 * (ranks.rank + 1)
        fake_t = {"mean_ms": wall * 1e3 / max(args.steps, 1), "launches": args.steps}
        fake_x = {"mean_ms": 0.01 * (ranks.rank + 1), "exchanges": args.warmup if ranks.world > 1 else 0,
                  "wait_ms": 0.004 * (ranks.rank + 1), "transfer_ms": 0.006 * (ranks.rank + 1)}
        per_rank = rank_stats(ranks, wall, fake_t, fake_x, {"nranks": ranks.world, "transport": "dry-run"})
        dt = ranks.max(wall)
        value, cfg, roof, dtype = 0.0, {"workload": "dry-run", "ranks": ranks.world}, None, None
        if ranks.world > 1:
            cfg["rank_stats"] = per_rank
    elif args.workload == "byte16k":
        value, dt, cfg, roof, dtype = run_bytes(args, ranks)
    else:
        value, dt, cfg, roof, dtype = run_bits(args, ranks)
    cpu = None
    if ranks.rank == 0 and ranks.world == 1 and not args.no_cpu_baseline and not args.dry_run:
        cpu = cpu_baseline(args)
    if ranks.rank == 0:
        line = {"metric": METRIC, "value": round(value / 1e9, 2), "unit": "GCUPS", "n_gpus": ranks.world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
                "higher_is_better": True, "scaling": "strong" if args.workload == "strong262k" else "weak",
                "vs_baseline": None, "dtype": dtype,
                "data": "synthetic (splitmix64 Bernoulli(1/2) torus generated on the GPU)",
                "config": cfg, "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    ranks.close()
    if cfg.get("parity", {}).get("status") == "FAIL":
        sys.exit(1)  # a board that differs from the reference is not a measurement


if __name__ == "__main__":
    main()
