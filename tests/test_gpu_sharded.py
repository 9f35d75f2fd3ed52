"""Row-sharded board with the real gfx950 kernels: several ranks share the one GPU of
the test box (gloo backend, halo rows staged through the host).  The production
multi-GPU path differs only in the transport (nccl = RCCL P2P over xGMI).

Checks every rank count gives the oracle's board (hash, counts) -- including uneven
shards and the interior/boundary launch split -- and equals the single-rank result."""
import os
import socket

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, H, W, k, turns, q, layout="auto"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "gol-distributed-final_amd")]
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golhip.sharded import ShardedBoard
        b = ShardedBoard(H, W, turns_per_launch=k, layout=layout)
        b.load_random(3)
        b.step(turns, count=True)
        torch.cuda.synchronize()
        q.put((rank, b.hash(), b.alive_count(), b.fused_count()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,W,k,turns", [(2, 1024, 64 * 40, 8, 37), (3, 1000, 64 * 40, 16, 50),
                                                (4, 515, 64 * 40, 4, 21),
                                                # W % 1024 == 0: band layout, halos are band rows
                                                (2, 1024, 2048, 8, 37), (3, 301, 3072, 4, 22),
                                                (2, 200, 4096, 12, 41)])
def test_sharded_gpu_ranks_match_oracle(world, H, W, k, turns):
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ref = O.bits_run(O.random_words(3, 0, H, W // 64), turns)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, k, turns, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, h, count, fused in res:
        assert h == O.hash_words(ref)
        assert count == fused == O.popcount_words(ref)


def _pgm_worker(rank, world, port, path, W, H, turns, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "gol-distributed-final_amd")]
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golhip.sharded import ShardedBoard
        b = ShardedBoard(H, W)
        b.load_pgm(path, chunk_rows=100)
        b.step(turns, count=True)
        torch.cuda.synchronize()
        full = b.gather_bytes()
        q.put((rank, b.fused_count(), full.numpy() if full is not None else None))
    finally:
        dist.destroy_process_group()


def _run_pgm(world, path, W, H, turns):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pgm_worker, args=(r, world, port, path, W, H, turns, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (c, full) for r, c, full in (q.get(timeout=150) for _ in range(world))}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


def test_sharded_gpu_load_pgm_golden(golden_dir):
    """Two ranks stream their rows of images/512x512.pgm into GPU shards; after 100 turns the
    gathered board is check/images/512x512x100.pgm."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_pgm(2, os.path.join(golden_dir, "images", "512x512.pgm"), 512, 512, 100)
    _, _, want = O.read_pgm(os.path.join(golden_dir, "check", "images", "512x512x100.pgm"))
    assert np.array_equal(res[0][1], want)
    assert res[0][0] == res[1][0] == int(np.count_nonzero(want))


def test_sharded_gpu_load_pgm_band(tmp_path):
    """A 2048-wide PGM (band layout, k = 12 split pipeline) streamed into 3 shards."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    H, W, turns = 150, 2048, 29
    rng = np.random.default_rng(5)
    board = (rng.random((H, W)) < 0.4).astype(np.uint8) * 255
    p = tmp_path / "b.pgm"
    p.write_bytes(O.pgm_bytes(board))
    res = _run_pgm(3, str(p), W, H, turns)
    ref = O.unpack(O.bits_run(O.pack(board), turns))
    assert np.array_equal(res[0][1], ref)


def _bench_line(args):
    """Run bench.py (it starts its own ranks for --gpus N > 1) and parse its JSON line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "bench.py"] + args, cwd=root, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_self_launch_two_replicas():
    """`python bench.py --gpus 2 --workload bit64k` with no launcher: the parent starts 2 ranks
    before touching the GPU; bit64k is a one-GPU workload, so each rank steps its own replica of
    the 65536^2 torus: the line must report 2x the one-rank alive count and the whole-job rate
    from the max-over-ranks time.  (The sharded workloads with --share-gpu run the rank engine
    over IPC: tests/test_gpu_ranks.py.)"""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    common = ["--workload", "bit64k", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--settle-s", "0"]
    two = _bench_line(["--gpus", "2", "--share-gpu"] + common)
    one = _bench_line(common)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["parallelism"] == "replicas2"
    assert two["config"]["turns_done"] == one["config"]["turns_done"]
    assert two["config"]["alive_final"] == 2 * one["config"]["alive_final"]
    k = one["config"]["turns_per_step"]
    assert abs(two["value"] - 2 * 65536 * 65536 * k * 3 / (two["ms_per_step"] * 3e-3) / 1e9) < 0.02 * two["value"]
    assert one["roofline"]["launch_ms"] > 0 and one["config"]["timed_launches"] == 3


def test_bench_settle_steps_reported():
    """The clock-settle phase (bench.py --settle-s; its default is the parser's): untimed steps before the
    warmup, a fixed count per workload (reproducible turns and counts), reported as
    config.settle_steps and counted in turns_done; the timed steps are exactly --steps launches."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    line = _bench_line(["--workload", "bit64k", "--steps", "4", "--warmup", "1", "--no-cpu-baseline", "--settle-s", "0.2"])
    cfg = line["config"]
    k = cfg["turns_per_step"]
    # a fixed count from the nominal rate: 0.2 s x 145e12 / (65536^2 x 12) ~ 562 steps of bit64k
    assert cfg["settle_steps"] == int(0.2 * 145e12 / (65536 * 65536 * k) + 0.5)
    assert cfg["turns_done"] == (cfg["settle_steps"] + 1 + 4) * k
    assert cfg["timed_launches"] == 4 and line["steps"] == 4 and line["warmup"] == 1
