"""Every BASELINE.json configuration at its own size, through golhip.Engine -- the engine
path bench.py times -- against the oracle.

The oracle cannot run boards of 2^32..2^40 cells, so the big boards are tori TILED with a
small random torus: a torus tiled with copies of a th x tw torus evolves exactly as the
small torus does (every neighbourhood is a neighbourhood of the small torus), so every
tile of the big board must equal the oracle's small-board result, bit for bit, and every
alive count must be the small count times the number of tiles.  Boards are loaded and read
as bit-packed rows (gol_engine_load_words / store_words).  The random bench board itself is
checked against a second, independent kernel family (the standard-layout k = 1 step).

  config 3  65536^2, k = 12 band pipeline (one round, paired ranges)    test_config3_*
  config 4  262144^2 on one GPU, and as 2 shards of that GPU            test_config4_*
  config 5  the bench's 2^17 x 2^20 per-GPU shard, exact bench workload test_config5_bench_*
            the whole 2^20 x 2^20 torus on one GPU, counts every 10
            turns and the P5 snapshot streamed to a sink                test_config5_full_*
(config 1 and 2 at size: tests/test_gpu_engine.py.)
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import golhip
    golhip.lib()
    return golhip


def _tile(seed, th, tw, turns, every):
    """A random th x tw torus (uint64 words) and the oracle's result and counts after `turns`."""
    words = O.random_words(seed, 0, th, tw // 64)
    ref, counts = O.bits_run(words, turns, with_counts=True)
    return words, ref, [int(c) for c in counts[every - 1::every]]


def _load_tiled(e, H, W, tile, chunk_rows=8192):
    th, tww = tile.shape
    assert H % th == 0 and W % (64 * tww) == 0 and chunk_rows % th == 0
    block = np.tile(tile, (chunk_rows // th, W // 64 // tww))
    for y in range(0, H, chunk_rows):
        n = min(chunk_rows, H - y)
        e.load_words(y, block[:n])


def _check_tiled(e, H, W, ref, chunk_rows=8192):
    th, tww = ref.shape
    for y in range(0, H, chunk_rows):
        n = min(chunk_rows, H - y)
        got = e.store_words(y, y + n).reshape(n // th, th, W // 64 // tww, tww)
        assert (got == ref[None, :, None, :]).all(), f"rows [{y}, {y + n})"


def _free_engine(e):
    import torch
    e.close()
    torch.cuda.empty_cache()


def test_config3_65536_tiled(G):
    """65536^2 (config 3): two k = 12 launches with the count fused into each (the bench's
    step), a 1-turn launch, then the whole board against the oracle's 256 x 1024 tile."""
    H = W = 65536
    tile, ref, counts = _tile(31, 256, 1024, 25, 12)
    reps = (H // 256) * (W // 1024)
    with G.Engine(H, W, device=0) as e:
        info = e.info()
        assert info["layout"] == "band" and info["turns_per_launch"] == 12
        _load_tiled(e, H, W, tile)
        got = e.step_counted(24, 12)
        assert got.tolist() == [reps * c for c in counts]
        e.step(1)
        _check_tiled(e, H, W, ref)
        assert e.alive_count() == reps * O.popcount_words(ref)


def test_config4_262144_full_board(G):
    """262144^2 (config 4) on one GPU (8 GiB per buffer): 24 turns in two counted k = 12
    launches, every tile against the oracle; then the same board as 2 row shards of the same
    GPU (loopback halo plan) gives the same hash and counts."""
    H = W = 262144
    tile, ref, counts = _tile(41, 512, 2048, 24, 12)
    reps = (H // 512) * (W // 2048)
    with G.Engine(H, W, device=0) as e:
        _load_tiled(e, H, W, tile)
        assert e.step_counted(24, 12).tolist() == [reps * c for c in counts]
        _check_tiled(e, H, W, ref, chunk_rows=16384)
        h1 = e.hash()
        _free_engine(e)
    with G.Engine(H, W, device=0, shards=2, same_device=True, transport="loopback") as e:
        _load_tiled(e, H, W, tile)
        assert e.step_counted(24, 12).tolist() == [reps * c for c in counts]
        assert e.hash() == h1
        _free_engine(e)


@pytest.mark.parametrize("H,W", [(65536, 262144), (32768, 262144), (131072, 262144)])
def test_config4_rank_shares_tiled(G, H, W):
    """Config 4's per-rank shares at N = 4, 8 and 2 (65536, 32768, 131072 rows x 262144): the
    first two run as one round of rank-weighted, paired ranges (the 65536-row share since round 4,
    GOL_BAND_RANK_ROUNDS), the third as 9 rounds of strips; through the serial and the overlapped
    step plan of a one-rank RCCL engine (the plan of the N-GPU run: ghost rows from the exchange,
    contiguous rows), counted every 12 turns, every tile against the oracle."""
    tile, ref, counts = _tile(43, 256, 1024, 36, 12)
    reps = (H // 256) * (W // 1024)
    for step in ("serial", "overlap"):
        with G.Engine.rank(H, W, 1, 0, G.engine.rccl_unique_id(), device=0, transport="rccl", step=step) as e:
            _load_tiled(e, H, W, tile)
            assert e.step_counted(36, 12).tolist() == [reps * c for c in counts]
            _check_tiled(e, H, W, ref, chunk_rows=16384)
            _free_engine(e)


@pytest.mark.timeout(300)
def test_config5_bench_workload_exact(G):
    """The driver's bench command exactly (`bench.py --gpus 1 --steps 20 --warmup 5`: seed 1,
    2^17 x 2^20, bench.py's own settle steps + 5 warmup + 20 timed k = 12 launches, the count fused
    into every launch), as a CROSS-KERNEL check: every count and the final hash of the band
    pipeline equal a run of the standard-layout k = 1 kernel (another kernel family, not an
    independent oracle) counted every 12 turns, and the last count is the `alive_final` of the
    driver's line (BENCH_r04.json: 6,080,808,203 at turn 936).  The settle count comes from
    bench.py itself, so a change of its settle rule or of a kernel that alters the driver's count
    fails here (count_test.go:44-51 pins counts per turn the same way).  At this size the oracle
    itself is too slow; the band pipeline is pinned to the oracle bit for bit by the tiled-torus
    tests at 65536^2, 262144^2 and 2^20 x 2^20 (below and above)."""
    import bench
    H, W, k = 1 << 17, 1 << 20, 12
    args = bench.parse(["--gpus", "1", "--steps", "20", "--warmup", "5"])
    calls = []
    settle = bench.settle_steps(args, calls.append, float(H) * W * k, bench.SETTLE_RATE_BITS)
    launches = settle + args.warmup + args.steps
    assert calls == [settle] and launches * k == 936, "the driver's turn count changed: re-pin alive_final"
    with G.Engine(H, W, device=0) as e:
        assert e.info()["turns_per_launch"] == k and e.info()["layout"] == "band"
        e.load_random(1)
        band = []
        for n in (settle, args.warmup, args.steps):  # bench.run_bits' three stepping calls
            band += e.step_counted(n * k, k).tolist()
        h_band = e.hash()
        _free_engine(e)
    with G.Engine(H, W, device=0, layout="standard", turns_per_launch=1) as e:
        assert e.info()["turns_per_launch"] == 1
        e.load_random(1)
        std = e.step_counted(launches * k, k).tolist()
        h_std = e.hash()
        _free_engine(e)
    assert band == std
    assert h_band == h_std
    assert band[24] == 8848272907  # BENCH_r02.json config.alive_final (turn 300)
    assert band[-1] == 6080808203  # BENCH_r04.json config.alive_final (turn 936)


@pytest.mark.timeout(600)
def test_config5_full_board_one_gpu(G):
    """The whole 2^20 x 2^20 torus of config 5 on ONE GPU (2 x 128 GiB of the 288 GB HBM): 30
    turns with the alive count every 10 turns (distributor.go:39-51's AliveCellsCount, fused on
    the GPU), every count against the oracle's tile, then the P5 snapshot (io.go:42-87, 1 TiB)
    streamed through gol_engine_write_pgm_to into a sink that checks the header, the offsets
    and every 97th chunk of rows byte for byte against the oracle's tile."""
    import torch
    H = W = 1 << 20
    th, tw = 256, 1024
    tile, ref, counts = _tile(51, th, tw, 30, 10)
    reps = (H // th) * (W // tw)
    try:
        e = G.Engine(H, W, device=0)
    except G.GolError as x:
        free, total = torch.cuda.mem_get_info(0)
        pytest.skip(f"2^20 x 2^20 does not fit: {x} (free {free / 2**30:.1f} of {total / 2**30:.1f} GiB)")
    try:
        _load_tiled(e, H, W, tile, chunk_rows=4096)
        assert e.step_counted(30, 10).tolist() == [reps * c for c in counts]
        assert e.alive_count() == reps * O.popcount_words(ref)
        ref_rows = O.unpack(ref)  # th x tw bytes, 0 / 255
        header = b"P5\n%d %d\n255\n" % (W, H)
        seen = {"next": 0, "chunks": 0, "checked": 0}

        def sink(off, buf):
            assert off == seen["next"], (off, seen["next"])
            n = len(buf)
            if off == 0:
                assert bytes(buf) == header
            else:
                assert (off - len(header)) % W == 0 and n % W == 0
                if seen["chunks"] % 97 == 0:
                    y = (off - len(header)) // W
                    got = np.frombuffer(buf, dtype=np.uint8).reshape(n // W, W // tw, tw)
                    want = ref_rows[np.arange(y, y + n // W) % th]
                    assert (got == want[:, None, :]).all(), f"rows at {y}"
                    seen["checked"] += 1
                seen["chunks"] += 1
            seen["next"] = off + n
        e.write_pgm_to(sink)
        assert seen["next"] == len(header) + H * W
        assert seen["checked"] > 100
    finally:
        _free_engine(e)


def _oracle_counts():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_counts.json")
    if not os.path.exists(path):
        return {}
    import json
    with open(path) as f:
        return json.load(f)["boards"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("key", sorted(_oracle_counts()))
def test_oracle_count_series(G, key):
    """The bench's random boards (`Engine.load_random(1)`, as bench.py loads them) at their full
    size, stepped on one GPU to the last turn the CPU oracle computed (tests/golden/oracle_counts.json,
    tools/pin_counts_oracle.py): every count -- the fused count of each launch -- and the final
    board's hash equal the oracle's (the hash once the oracle's series is complete).  Config 2's 16384^2 board runs on the byte board the byte16k
    line times (`layout="bytes"`, k = 32), the others on the bit board (k = 12)."""
    rec = _oracle_counts()[key]
    H, W, every, turns = rec["H"], rec["W"], rec["every"], rec["turns"]
    assert turns == every * len(rec["counts"]) and turns > 0
    layout = "bytes" if key == "16384x16384" else None
    kw = {"layout": layout} if layout else {}
    with G.Engine(H, W, device=0, **kw) as e:
        assert e.info()["turns_per_launch"] == (32 if layout else 12)
        e.load_random(1)
        counts = []
        chunk = every * 500
        while len(counts) * every < turns:
            n = min(chunk, turns - len(counts) * every)
            counts += [int(c) for c in e.step_counted(n, every)]
        assert counts == rec["counts"]
        if rec["hash_final"] is None:  # (a series the script has not finished: its counts only)
            return
        if layout:
            h = O.hash_words(O.pack(e.store_bytes()))
        else:
            h = e.hash()
    assert h == rec["hash_final"]
