"""Benchmark of the Game-of-Life hot path on MI355X (BASELINE.json metric:
cell-updates/s (GCUPS) and % of the HBM roofline at 1/2/4/8 GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload weak|bit64k|byte16k]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workloads (a "step" = one pass of the hot path = one k-turn launch over the board):
  weak     (default) bit-packed torus of 2^17 rows x 2^20 columns PER GPU, rows sharded
           over the ranks with a k-row RCCL halo exchange (SURVEY.md §8(d) weak-scaling
           config; N = 8 is the 2^20 x 2^20 torus of BASELINE.json config 5).
  strong262k  262144 x 262144 bit-packed torus, rows sharded over the N ranks (config 4:
           total work fixed as N grows, "scaling": "strong").
  bit64k   65536 x 65536 bit-packed torus on one GPU (config 3); replicas for N > 1.
  byte16k  16384 x 16384 byte-per-cell torus, 1 turn per step (config 2); replicas for N > 1.

Inputs are synthetic (splitmix64 Bernoulli(1/2) cells, generated on the GPU) and
resident in HBM before timing.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "gol-distributed-final_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
BITS_BYTES_PER_UPDATE = 0.25  # 1 bit read + 1 bit written per cell per turn
BYTES_BYTES_PER_UPDATE = 2.0  # 1 byte read + 1 byte written


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="weak", choices=["weak", "strong262k", "bit64k", "byte16k"])
    ap.add_argument("--k", type=int, default=0,
                    help="turns per launch (temporal blocking); 0 = library default for bit boards "
                         "(12 band / 8 standard), 32 for byte16k")
    ap.add_argument("--cpl", type=int, default=0, help="cells per lane (32/64/128; 0 = library default)")
    ap.add_argument("--strip", type=int, default=0, help="rows per wave strip (0 = auto)")
    ap.add_argument("--layout", default="auto", choices=["auto", "standard", "band"],
                    help="bit layout while stepping (auto = band when W %% 1024 == 0; DESIGN.md §4.1)")
    ap.add_argument("--rows-per-gpu", type=int, default=1 << 17)
    ap.add_argument("--width", type=int, default=1 << 20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU baseline sample length")
    ap.add_argument("--no-count", action="store_true",
                    help="do not fuse the alive-cell count (AliveCellsCount) into every launch")
    ap.add_argument("--snapshot-rows", type=int, default=0,
                    help="after the timed steps, stream this many board rows per rank as P5 bytes "
                         "(device unpack -> host, golhip.sharded.stream_pgm's path) and report the rate "
                         "(config 5's PGM snapshot; not part of value)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="testing only: every rank uses cuda:0 (multi-rank logic on a 1-GPU box, with --backend gloo)")
    return ap.parse_args()


def setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.share_gpu:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    return rank, world, local


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


class KernelTimer:
    """HIP events around every launch of one kind, on the stream the kernel runs on."""

    def __init__(self, kinds):
        self.kinds = set(kinds)
        self.pairs = []
        self.enabled = False
        self._open = None

    def __call__(self, kind, k, rows, before):
        if not self.enabled or kind not in self.kinds:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream())
        if before:
            self._open = (ev, k, rows)
        else:
            s, kk, rr = self._open
            self.pairs.append((s, ev, kk, rr))

    def avg(self):
        ms = [s.elapsed_time(e) for s, e, _, _ in self.pairs]
        return sum(ms) / len(ms), self.pairs[0][2], self.pairs[0][3]


def cpu_baseline(args, H, W, k):
    """Oracle restatement of the reference (literal worker.go port, one pthread per slab as the
    broker's workers) on the host cores; bounded sample of the same synthetic board."""
    from oracle import oracle as O
    threads = min(16, os.cpu_count() or 1)
    side = 1024
    words = O.random_words(1, 0, side, side // 64)
    board = O.unpack(words)
    t0 = time.perf_counter()
    O.run(board, 1, threads)
    one = max(time.perf_counter() - t0, 1e-4)
    turns = max(1, int(args.cpu_seconds / one))
    t0 = time.perf_counter()
    O.run(board, turns, threads)
    dt = time.perf_counter() - t0
    return {"value": side * side * turns / dt / 1e9, "unit": "GCUPS", "cores": threads, "kind": "port",
            "sample": f"{side}x{side} torus (same splitmix64 board generator), {turns} turns, literal per-cell "
                      f"port of worker.go:15-70 with the broker's {threads}-slab split (oracle/gol_oracle.c); "
                      f"the Go reference cannot be built here"}


def load_pmc(key):
    """Measured HBM bytes per launch for this exact configuration (tools/pmc_summary.py)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(key)
    except (OSError, ValueError):
        return None


def run_bits(args, rank, world):
    from golhip.sharded import ShardedBoard
    if args.workload == "weak":
        H, W, nshards = args.rows_per_gpu * world, args.width, world
    elif args.workload == "strong262k":
        H, W, nshards = 262144, 262144, world
    else:
        H, W, nshards = 65536, 65536, 1
    group = None
    if nshards == 1 and world > 1:  # independent replicas: every rank its own board, no collective
        group = [dist.new_group([r]) for r in range(world)][rank]
    board = ShardedBoard(H, W, turns_per_launch=args.k, cells_per_lane=args.cpl, strip_rows=args.strip,
                         group=group, layout=args.layout)
    layout = "band" if board.use_band else "standard"
    k = board.kmax
    board.load_random(1)
    timer = KernelTimer(["full", "interior"])
    board.launch_hook = timer
    count = not args.no_count  # AliveCellsCount fused into the last generation of every launch
    for _ in range(args.warmup):
        board.step(k, count=count)
    barrier(world)
    timer.enabled = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        board.step(k, count=count)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    barrier(world)
    timer.enabled = False
    dt = max_over_ranks(dt, world)
    alive = board.fused_count() if count else None
    cells_total = H * W * (world if nshards == 1 else 1)
    value = cells_total * k * args.steps / dt
    kms, kk, krows = timer.avg()
    alg_bytes = BITS_BYTES_PER_UPDATE * krows * W * kk
    achieved = alg_bytes / (kms * 1e-3) / 1e9
    from golhip import lib
    info = {"turns_per_step": k, "layout": layout,
            "cells_per_lane": 128 if layout == "band" else (args.cpl or "lib default (64)"),
            "strip_rows": args.strip or "auto",
            "alive_count_every_step": count, "alive_final": alive, "turns_done": board.turn}
    pmc = load_pmc(f"{args.workload}:{H}x{W}:n{world}:k{k}:" + ("band" if layout == "band" else f"cpl{args.cpl}"))
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc.get("bytes_per_launch") if pmc else None,
            # with k turns per launch the kernel is bound by VALU issue, not HBM:
            # the PMC-measured share of the 2-cycle VALU issue peak, from the same profile
            "valu_issue_frac": pmc.get("valu_issue_frac") if pmc else None,
            "basis": f"{BITS_BYTES_PER_UPDATE} B/cell-update x {krows}x{W} cells x {kk} turns per launch "
                     f"/ {kms:.3f} ms mean launch ({len(timer.pairs)} launches, HIP events)",
            "hbm_min_bytes_frac": round(2 * krows * W / 8 / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    del lib
    rpg = args.rows_per_gpu
    rows_name = f"2^{rpg.bit_length() - 1}" if rpg & (rpg - 1) == 0 else str(rpg)
    wname = f"2^{W.bit_length() - 1}" if W & (W - 1) == 0 else str(W)
    snap = snapshot(board, args.snapshot_rows, world) if args.snapshot_rows > 0 else None
    name = {"weak": f"weak-{rows_name}x{wname}-per-gpu", "strong262k": "strong-262144x262144",
            "bit64k": "bit-65536x65536"}[args.workload]
    cfg = {"workload": name,
           "H": H, "W": W, "parallelism": (f"rows{world}" if nshards > 1 else (f"replicas{world}" if world > 1 else "1gpu")),
           **info}
    if snap is not None:
        cfg["snapshot"] = snap
    dtype = "u32 (bit-packed, 32 cells/word" + (", column-band layout)" if layout == "band" else ")")
    return value, dt, cfg, roof, dtype


def snapshot(board, rows, world):
    """Config 5's PGM snapshot path, bounded: every rank unpacks its first `rows` rows on the GPU
    (bits -> 0/255 bytes, golhip.sharded.stream_pgm's chunked path) and copies them to the host;
    reported as host bytes/s over all ranks (PCIe-inclusive, not part of value)."""
    rows = min(rows, board.R)
    std = board.standard()
    chunk = 4096
    barrier(world)
    t0 = time.perf_counter()
    n = 0
    for a in range(0, rows, chunk):
        part = board.kern.unpack(std[a:a + min(chunk, rows - a)], board.W)
        n += part.cpu().numpy().nbytes
    torch.cuda.synchronize()
    dt = max_over_ranks(time.perf_counter() - t0, world)
    return {"rows_per_rank": rows, "bytes": n * world, "GB_per_s": round(n * world / dt / 1e9, 2)}


def run_bytes(args, rank, world):
    """Config 2: 16384 x 16384 byte-per-cell torus.  The board stays one byte per cell in HBM;
    with --k > 1 each launch runs k turns (gol_dev_bytes_step_k: 0/255 bytes packed to bits in
    registers), with --k 1 the exact one-turn byte kernel (gol_dev_bytes_step)."""
    from golhip._lib import check, lib
    from golhip.sharded import HipKernels
    H = W = 16384
    Wd = W // 32
    bits = torch.empty((H, Wd), dtype=torch.int32, device="cuda")
    kern = HipKernels()
    kern.Wd = Wd
    kern.random_fill(bits, 0, W, 1)
    a = kern.unpack(bits, W)
    b = torch.empty_like(a)
    del bits
    stream = torch.cuda.current_stream().cuda_stream
    k = max(kk for kk in (32, 16, 8, 4, 2, 1) if kk <= args.k)
    pairs = []
    cur = [a, b]

    def step(timed):
        src, dst = cur
        if timed:
            s = torch.cuda.Event(enable_timing=True)
            s.record()
        if k == 1:
            check(lib().gol_dev_bytes_step(src.data_ptr(), H, W, W, 0, H, dst.data_ptr(), W, stream))
        else:
            check(lib().gol_dev_bytes_step_k(src[H - k:].data_ptr(), src.data_ptr(), src.data_ptr(), dst.data_ptr(),
                                             H, W, W, 0, H, k, args.strip, None, stream))
        if timed:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            pairs.append((s, e))
        cur.reverse()

    for _ in range(args.warmup):
        step(False)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    barrier(world)
    dt = max_over_ranks(dt, world)
    value = H * W * world * k * args.steps / dt
    kms = sum(s.elapsed_time(e) for s, e in pairs) / len(pairs)
    achieved = BYTES_BYTES_PER_UPDATE * H * W * k / (kms * 1e-3) / 1e9
    pmc = load_pmc(f"byte16k:{H}x{W}:n1:k{k}:cpl0")
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc.get("bytes_per_launch") if pmc else None,
            "basis": f"{BYTES_BYTES_PER_UPDATE} B/cell-update x {H}x{W} cells x {k} turns per launch / "
                     f"{kms:.3f} ms mean launch",
            "hbm_min_bytes_frac": round(2 * H * W / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    cfg = {"workload": "byte-16384x16384", "H": H, "W": W, "turns_per_step": k,
           "parallelism": f"replicas{world}" if world > 1 else "1gpu"}
    return value, dt, cfg, roof, "u8 (byte per cell)"


def main():
    args = parse()
    if args.k <= 0 and args.workload == "byte16k":
        args.k = 32  # pipelined byte kernel, 8 waves x 4 turns; bit boards: 0 = library default (12 on the band layout, 8 on the standard one)
    rank, world, local = setup(args)
    if args.workload == "byte16k":
        value, dt, cfg, roof, dtype = run_bytes(args, rank, world)
    else:
        value, dt, cfg, roof, dtype = run_bits(args, rank, world)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, cfg["H"], cfg["W"], cfg.get("turns_per_step", 1))
    if rank == 0:
        line = {"metric": "cell-updates/sec (GCUPS) + % HBM roofline at 1/2/4/8 MI355X", "value": round(value / 1e9, 2),
                "unit": "GCUPS", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
                "scaling": "strong" if args.workload == "strong262k" else "weak", "vs_baseline": None,
                "dtype": dtype,
                "data": "synthetic (splitmix64 Bernoulli(1/2) torus generated on the GPU)",
                "config": cfg, "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
