"""GPU parity of the row-sharded engine behind the C ABI (gol_engine_create with
gol_config.shards, gol_engine_create_rank).

The reference splits the board into `Threads` row slabs (broker.go:135-206) and
ships the whole board to every worker each turn; the engine applies the same
split to GPUs once and exchanges k halo rows per launch.  On the one-GPU test
box several shards share cuda:0 with the LOOPBACK transport (device copies),
and the RCCL code path runs with one shard sending its halo to itself.  Every
result is compared with the oracle (or the single-GPU engine at sizes the
oracle cannot run), bit-exact.
"""
import ctypes
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def G():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import golhip
    golhip.lib()
    return golhip


def _sharded(G, H, W, n, **kw):
    kw.setdefault("device", 0)
    return G.Engine(H, W, shards=n, same_device=True, transport=kw.pop("transport", "loopback"), **kw)


@pytest.mark.parametrize("n", [1, 2, 3, 4])
@pytest.mark.parametrize("H,W,layout", [(203, 2048, "band"), (97, 64 * 9, "standard"), (130, 4096, "standard")])
def test_loopback_shards_vs_oracle(G, n, H, W, layout):
    """N = 1..4 shards on uneven splits (203 = 51+51+51+50 rows ...): hash, bytes, count."""
    seed = 7 * n + W
    words = O.random_words(seed, 0, H, W // 64)
    ref, counts = O.bits_run(words, 45, with_counts=True)
    with _sharded(G, H, W, n, layout=layout) as e:
        topo = e.topology()
        assert topo["shards"] == n and topo["nranks"] == n and topo["transport"] == "loopback"
        for i in range(n):
            assert (e.shard(i)["y0"], e.shard(i)["y1"]) == O.partition(H, n, i)
        e.load_random(seed)
        assert e.hash() == O.hash_words(words)
        e.step(20)
        assert e.alive_count() == counts[19]
        e.step(25)
        assert e.hash() == O.hash_words(ref)
        assert np.array_equal(e.store_bytes(), O.unpack(ref))
        assert e.alive_count() == O.popcount_words(ref)


@pytest.mark.parametrize("H,n,W,layout", [(9, 4, 1024, "band"), (5, 3, 2048, "band"), (4, 4, 1024, "band"),
                                           (7, 3, 128, "standard"), (3, 3, 64, "standard")])
def test_tiny_shards_cap_turns_per_launch(G, H, n, W, layout):
    """Shards of 1-3 rows: the engine caps k at the smallest shard (the halo exchange hands over
    k rows of ONE neighbour), so every launch is exact; 29 turns against the oracle."""
    seed = 100 + H * n
    words = O.random_words(seed, 0, H, W // 64)
    ref, counts = O.bits_run(words, 29, with_counts=True)
    with _sharded(G, H, W, n, layout=layout) as e:
        assert [e.shard(i)["y1"] - e.shard(i)["y0"] for i in range(n)] == \
            [O.partition(H, n, i)[1] - O.partition(H, n, i)[0] for i in range(n)]
        e.load_random(seed)
        assert e.step_counted(29, 1).tolist() == list(counts[:29])
        assert e.hash() == O.hash_words(ref)


@pytest.mark.parametrize("n", [2, 3])
def test_concurrent_shards_paired_ranges(G, n):
    """Shards on one GPU launch on their own streams at once; each launch of a narrow band board
    takes the one-round rank split with paired ranges and its own claim counters.  Counted steps
    (the first launch of every fresh stream included) and the board against the oracle."""
    H, W = 65536 * n, 2048
    words = O.random_words(21 + n, 0, H, W // 64)
    ref, counts = O.bits_run(words, 36, with_counts=True)
    with _sharded(G, H, W, n) as e:
        e.load_random(21 + n)
        assert e.step_counted(36, 12).tolist() == [counts[11], counts[23], counts[35]]
        assert e.hash() == O.hash_words(ref)


def test_engines_in_sequence_reuse_streams(G):
    """Engines created and destroyed one after another (a new engine may get a destroyed one's
    stream handle, and with it that stream's claim counters): the first counted launch of each is
    exact, for band boards of 1, 2, 1 and 4 column groups."""
    for H, W, seed in ((65536, 2048, 1), (32768, 4096, 2), (65536, 1024, 3), (16384, 8192, 4)):
        words = O.random_words(seed, 0, H, W // 64)
        ref, counts = O.bits_run(words, 12, with_counts=True)
        with G.Engine(H, W, device=0) as e:
            e.load_random(seed)
            assert e.step_counted(12, 12).tolist() == [counts[11]], (H, W)
            assert e.hash() == O.hash_words(ref), (H, W)


@pytest.mark.parametrize("H,W", [(16, 16), (33, 32), (20, 48), (9, 8)])
def test_narrow_boards_byte_path(G, H, W):
    """Widths below 64 (or not a multiple of 64) run on the exact byte board: vs the literal port."""
    rng = np.random.default_rng(H * W)
    board = (rng.random((H, W)) < 0.4).astype(np.uint8) * 255
    with G.Engine(H, W, device=0) as e:
        e.load_bytes(board)
        counts = e.step_counted(23, 1)
        got = e.store_bytes()
    ref = board
    want = []
    for _ in range(23):
        ref = O.run(ref, 1)
        want.append(int(np.count_nonzero(ref)))
    assert np.array_equal(got, ref)
    assert counts.tolist() == want


@pytest.mark.parametrize("n", [2, 3])
def test_shards_bytes_golden_alive_list_pgm(G, golden_dir, tmp_path, n):
    """TestGol / TestPgm on the 512x512 golden board through a sharded engine: alive list in
    row-major order across shards, PGM written shard by shard byte-identical to check/images."""
    _, _, board = O.read_pgm(os.path.join(golden_dir, "images", "512x512.pgm"), 512, 512)
    with _sharded(G, 512, 512, n) as e:
        e.load_bytes(board)
        e.step(100)
        out = tmp_path / "512x512x100.pgm"
        e.write_pgm(str(out))
        cells = [tuple(c) for c in e.alive_cells().tolist()]
    gold = open(os.path.join(golden_dir, "check", "images", "512x512x100.pgm"), "rb").read()
    assert out.read_bytes() == gold
    ys, xs = np.nonzero(O.read_pgm(os.path.join(golden_dir, "check", "images", "512x512x100.pgm"))[2])
    assert cells == list(zip(xs.tolist(), ys.tolist()))


@pytest.mark.parametrize("n", [2, 4])
def test_shards_alive_csv_counted(G, golden_dir, n):
    """TestAlive's counts (check/alive/512x512.csv) from step_counted on a sharded board: the
    count fused into the launch ending every `every` turns, reduced on the device."""
    expected = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", "512x512.csv"))
    _, _, board = O.read_pgm(os.path.join(golden_dir, "images", "512x512.pgm"), 512, 512)
    with _sharded(G, 512, 512, n) as e:
        e.load_bytes(board)
        for every in (1, 7, 10, 12, 25):
            t0 = e.turn
            got = e.step_counted(10 * every + 3, every)
            assert e.turn == t0 + 10 * every + 3
            want = [expected[t0 + (i + 1) * every] for i in range((10 * every + 3) // every)]
            assert got.tolist() == want, f"every {every}"


def test_shards_non_binary_first_turn(G):
    """worker.go:26-37 with shards: each shard runs the exact byte turn over its rows plus the two
    halo rows it loaded from the host board."""
    rng = np.random.default_rng(5)
    H, W = 90, 128
    board = rng.choice(np.array([0, 255, 1, 7, 128], dtype=np.uint8), size=(H, W), p=[.5, .35, .05, .05, .05])
    with _sharded(G, H, W, 3) as e:
        e.load_bytes(board)
        assert np.array_equal(e.store_bytes(), board)
        assert e.alive_count() == int(np.count_nonzero(board))
        assert [tuple(c) for c in e.alive_cells().tolist()] == O.alive_cells(board)
        e.step(1)
        assert np.array_equal(e.store_bytes(), O.run(board, 1))
        e.step(12)
        assert np.array_equal(e.store_bytes(), O.run(board, 13))


def test_shards_step_flips(G):
    H, W = 75, 1024
    rng = np.random.default_rng(2)
    board = (rng.random((H, W)) < 0.35).astype(np.uint8) * 255
    with _sharded(G, H, W, 3) as e:
        e.load_bytes(board)
        e.step(12)
        prev = O.run(board, 12)
        for t in range(1, 4):
            got = [tuple(c) for c in e.step_flips().tolist()]
            cur = O.run(board, 12 + t)
            assert got == O.flipped_cells(prev, cur)
            prev = cur


def test_shards_load_pgm(G, golden_dir):
    """readPgmImage (gol/io.go:90-126) streamed per shard: every shard reads its own rows."""
    path = os.path.join(golden_dir, "images", "512x512.pgm")
    _, _, board = O.read_pgm(path, 512, 512)
    for n in (1, 3):
        with _sharded(G, 512, 512, n) as e:
            e.load_pgm(path)
            assert np.array_equal(e.store_bytes(), board)
            e.step(100)
            gold = O.read_pgm(os.path.join(golden_dir, "check", "images", "512x512x100.pgm"))[2]
            assert np.array_equal(e.store_bytes(), gold)
    with G.Engine(512, 512, device=0) as e:
        with pytest.raises(G.GolError, match="Incorrect width"):
            G.Engine(512, 256, device=0).load_pgm(path)
        e.load_pgm(path)
        assert np.array_equal(e.store_bytes(), board)


def test_load_pgm_fields_rules(G, tmp_path):
    """io.go:98-119 (strings.Fields): whitespace after maxval is skipped; a raster holding a
    whitespace byte is rejected; bytes other than 0/255 get the exact first turn."""
    rng = np.random.default_rng(4)
    H, W = 40, 128
    board = rng.choice(np.array([0, 255, 7], dtype=np.uint8), size=(H, W), p=[.5, .4, .1])
    p = tmp_path / "b.pgm"
    p.write_bytes(b"P5\n%d %d\n255\r\n" % (W, H) + board.tobytes())
    for n in (1, 2):
        with _sharded(G, H, W, n) as e:
            e.load_pgm(str(p))
            assert np.array_equal(e.store_bytes(), board)
            e.step(3)
            assert np.array_equal(e.store_bytes(), O.run(board, 3))
    ws = board.copy()
    ws[20, 5] = 32
    p.write_bytes(b"P5\n%d %d\n255\n" % (W, H) + ws.tobytes())
    with _sharded(G, H, W, 2) as e:
        with pytest.raises(G.GolError, match="whitespace"):
            e.load_pgm(str(p))


def test_rccl_transport_self(G):
    """The RCCL halo path on one GPU: one shard whose ncclSend/ncclRecv go to itself (the torus
    wrap), in-process (ncclCommInitAll) and as a one-rank Engine.rank (ncclCommInitRank)."""
    H, W = 150, 2048
    words = O.random_words(3, 0, H, W // 64)
    ref, counts = O.bits_run(words, 40, with_counts=True)
    with G.Engine(H, W, device=0, transport="rccl") as e:
        assert e.topology()["transport"] == "rccl"
        e.load_random(3)
        got = e.step_counted(40, 8)
        assert got.tolist() == [counts[8 * i + 7] for i in range(5)]
        assert e.hash() == O.hash_words(ref)
    uid = G.engine.rccl_unique_id()
    with G.Engine.rank(H, W, 1, 0, uid, device=0, transport="rccl") as e:
        assert e.topology() == {"shards": 1, "nranks": 1, "rank": 0, "transport": "rccl"}
        e.load_random(3)
        e.step(40)
        assert e.hash() == O.hash_words(ref)
        assert np.array_equal(e.store_rows(10, 20), O.unpack(ref)[10:20])


@pytest.mark.parametrize("step", ["serial", "overlap"])
def test_rccl_exchange_timing_self(G, step):
    """The timed RCCL exchange (ABI 6, what bench.py's N > 1 warmup runs on every rank): a one-word
    send/recv with each ring neighbour ahead of the halo group, here a one-rank Engine.rank whose
    neighbour is itself, on the compute stream after SERIAL steps and on the comm stream after
    OVERLAP ones.  The board is the oracle's, every exchange is timed, and the wait and the
    transfer add up to the whole."""
    H, W, k = 1000, 2048, 12
    ref, counts = O.bits_run(O.random_words(5, 0, H, W // 64), 60, with_counts=True)
    with G.Engine.rank(H, W, 1, 0, G.engine.rccl_unique_id(), device=0, transport="rccl", step=step) as e:
        e.load_random(5)
        e.set_timing(True, exchanges=True)
        got = e.step_counted(60, k)
        x = e.exchange_timing()
        e.set_timing(False)
        assert got.tolist() == [int(counts[k * (i + 1) - 1]) for i in range(5)]
        assert e.hash() == O.hash_words(ref)
    assert x["exchanges"] >= 5 and x["mean_ms"] > 0
    assert 0 <= x["wait_ms"] and 0 <= x["transfer_ms"] and abs(x["wait_ms"] + x["transfer_ms"] - x["mean_ms"]) < 1e-9


def test_broker_run_sharded(G, golden_dir):
    """Operations.Run with the board sharded over 3 shards (Threads 1..16 as in TestGol): the
    same alive list and board as check/images; the 16x16 board (W % 64 != 0) runs unsharded."""
    for size in (16, 64, 512):
        _, _, board = O.read_pgm(os.path.join(golden_dir, "images", f"{size}x{size}.pgm"), size, size)
        gold = O.read_pgm(os.path.join(golden_dir, "check", "images", f"{size}x{size}x100.pgm"))[2]
        ops = G.Operations(device=0, shards=3, transport="loopback", same_device=True)
        for threads in (1, 4, 16):
            res = ops.Run(G.Request(World=board, Turns=100, ImageHeight=size, ImageWidth=size, Threads=threads))
            assert np.array_equal(res.World, gold)
            ys, xs = np.nonzero(gold)
            assert [(c.X, c.Y) for c in res.Alive] == list(zip(xs.tolist(), ys.tolist()))
        ops.close()


def test_config4_width_sharded(G):
    """Config 4's width (262144 columns, band layout) row-sharded over 2 and 3 shards: the board is
    a torus tiled with a 1024-wide tile, so every tile must evolve like the oracle's small torus."""
    th, tw, H, W, turns = 64, 1024, 384, 262144, 30
    rng = np.random.default_rng(44)
    tile = (rng.random((th, tw)) < 0.4).astype(np.uint8) * 255
    ref = O.unpack(O.bits_run(O.pack(tile), turns))
    big = np.tile(tile, (H // th, W // tw))
    for n in (2, 3):
        with _sharded(G, H, W, n) as e:
            e.load_bytes(big)
            e.step(turns)
            assert e.info()["layout"] == "band"
            got = e.store_bytes().reshape(H // th, th, W // tw, tw)
            assert (got == ref[None, :, None, :]).all()


def test_config5_periodic_count_and_snapshot(G, tmp_path):
    """Config 5's pieces on a sharded board: the alive count every 10 turns (fused, on the GPU)
    equals a per-turn popcount of a second run, and the P5 snapshot written shard by shard equals
    the single-GPU engine's file (sha256), at 4096 x 65536; and both equal the oracle on a small
    board."""
    H, W, turns = 4096, 65536, 120
    with _sharded(G, H, W, 4) as e:
        e.load_random(9)
        periodic = e.step_counted(turns, 10)
        snap = tmp_path / "sharded.pgm"
        e.write_pgm(str(snap))
        h_sharded = e.hash()
    per_turn = []
    with G.Engine(H, W, device=0) as e:
        e.load_random(9)
        for _ in range(turns):
            e.step(1)
            per_turn.append(e.alive_count())
        one = tmp_path / "one.pgm"
        e.write_pgm(str(one))
        assert e.hash() == h_sharded
    assert periodic.tolist() == per_turn[9::10]
    digest = lambda p: hashlib.sha256(p.read_bytes()).hexdigest()  # noqa: E731
    assert digest(snap) == digest(one)
    # small board: the same calls against the oracle
    words = O.random_words(9, 0, 300, 16)
    ref, counts = O.bits_run(words, 60, with_counts=True)
    with _sharded(G, 300, 1024, 4) as e:
        e.load_random(9)
        assert e.step_counted(60, 10).tolist() == counts[9::10].tolist()
        e.write_pgm(str(tmp_path / "small.pgm"))
    assert (tmp_path / "small.pgm").read_bytes() == O.pgm_bytes(O.unpack(ref))


def test_timing_counts_the_step_launches(G):
    with _sharded(G, 600, 2048, 2) as e:
        e.load_random(1)
        e.set_timing(True)
        e.step(36)  # 3 steps of k = 12 on each of the 2 shards, every launch of a step inside its timing
        t = e.timing()
        assert t["launches"] == 6 and t["mean_ms"] > 0
        assert t["mean_cell_updates"] == 300 * 2048 * 12


def test_timing_many_exchanges_in_one_call(G):
    """one timed call with more exchanges than the event pool holds (2 loopback shards,
    300 exchanges of 4 events per shard against a pool of 512).  The pool grows inside the call
    instead of being folded while the call's own start event is live, so the call's step time is
    the same as with exchange timing off, every exchange is counted, and the loopback exchange
    (no peer in another process) waits for nothing.  The board is the oracle's either way."""
    H, W, k, steps = 64, 1024, 4, 300
    res = {}
    for x in (False, True):
        with _sharded(G, H, W, 2, turns_per_launch=k) as e:
            e.load_random(4)
            e.step(12 * k)  # (clocks, allocations)
            e.set_timing(True, exchanges=x)
            e.step(steps * k)
            t, xt = e.timing(), e.exchange_timing()
            e.set_timing(False)
            res[x] = (t, xt, e.hash())
    ref = O.bits_run(O.random_words(4, 0, H, W // 64), (12 + steps) * k)
    for t, xt, h in res.values():
        assert h == O.hash_words(ref)
        assert t["launches"] == 2 * steps and t["mean_cell_updates"] == 32 * W * k
    t0, x0, _ = res[False]
    t1, x1, _ = res[True]
    assert x0["exchanges"] == 0
    assert x1["exchanges"] >= 2 * steps and x1["mean_ms"] > 0
    # (two events recorded back to back on a stream still read ~10 us apart)
    assert 0 <= x1["wait_ms"] < 0.05 and abs(x1["wait_ms"] + x1["transfer_ms"] - x1["mean_ms"]) < 1e-9
    assert 0.5 < t1["mean_ms"] / t0["mean_ms"] < 2.0, (t0, t1)


def test_timing_then_flips_outside_a_timed_call(G):
    """with timing on, a step_flips call (not a timed stepping call) must not write the
    per-call timing arrays (it used to index them out of bounds when no step had run) and must not
    count as a timed step."""
    H, W = 200, 2048
    words = O.random_words(2, 0, H, W // 64)
    with G.Engine(H, W, device=0) as e:
        e.load_random(2)
        e.set_timing(True)
        flips = e.step_flips()
        assert e.timing()["launches"] == 0
        e.step(12)
        assert e.timing()["launches"] == 1
        ref1 = O.bits_run(words, 1)
        want = O.flipped_cells(O.unpack(words), O.unpack(ref1))
        assert [tuple(x) for x in flips.tolist()] == [tuple(x) for x in want]
        assert e.hash() == O.hash_words(O.bits_run(ref1, 12))


def test_device_fault_is_reported(G):
    """A pipeline wave that gives up waiting (the test build libgolhip_spintest.so times out every
    flag wait at once) must surface as GOL_EHIP, not as a board with unwritten strips (child
    process: a second build of the library)."""
    spin = os.path.join(ROOT, "gol-distributed-final_amd", "golhip", "libgolhip_spintest.so")
    if not os.path.exists(spin):
        pytest.skip("libgolhip_spintest.so not built (make -C gol-distributed-final_amd/csrc spintest)")
    code = (
        "import sys, ctypes; sys.path[:0] = [%r, %r]\n"
        "import golhip, golhip._lib as L\n"
        "lib = L.load(%r)\n"
        "for shape in ((200, 2048), (150, 1024)):\n"
        "    e = golhip.Engine(*shape, device=0, library=lib)\n"
        "    e.load_random(1)\n"
        "    try:\n"
        "        e.step(24)\n"
        "        raise SystemExit('no error')\n"
        "    except golhip.GolError as x:\n"
        "        assert x.code == L.GOL_EHIP and 'timed out' in str(x), x\n"
        "    e.step(1)  # the error word was cleared; k = 1 has no flag waits\n"
        "    e.close()\n"
        "print('ok')\n" % (ROOT, os.path.join(ROOT, "gol-distributed-final_amd"), spin))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]
    # the product library reports no fault for the same calls
    with G.Engine(200, 2048, device=0) as e:
        e.load_random(1)
        e.step(24)
    flags = ctypes.c_uint32()
    assert G.lib().gol_dev_error(0, ctypes.byref(flags)) == 0 and flags.value == 0
