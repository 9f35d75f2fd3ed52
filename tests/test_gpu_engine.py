"""GPU parity tests: libgolhip.so (gfx950 kernels) against the oracle and the
reference's golden fixtures.  Every call goes through the C ABI.

Mirrors the reference's end-to-end tests:
  TestGol   gol_test.go:15-47     -> test_gol_matrix (sizes x turns x threads 1..16)
  TestPgm   pgm_test.go:10-42     -> test_pgm_output
  TestAlive count_test.go:17-69   -> test_alive_counts_csv / test_alive_parity_rule
plus size-independent properties at the bench's full size.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [16, 64, 512]
TURNS = [0, 1, 100]


@pytest.fixture(scope="module")
def golhip():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import golhip as G
    G.lib()
    return G


def _golden_board(golden_dir, size):
    return O.read_pgm(os.path.join(golden_dir, "images", f"{size}x{size}.pgm"), size, size)[2]


def _golden_alive(golden_dir, size, turns):
    """gol_test.go:88-129 readAliveCells: every nonzero byte of the golden PGM is alive."""
    _, _, g = O.read_pgm(os.path.join(golden_dir, "check", "images", f"{size}x{size}x{turns}.pgm"))
    ys, xs = np.nonzero(g)
    return set(zip(xs.tolist(), ys.tolist())), g


# ------------------------------------------------------------------ reference test matrix
@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("turns", TURNS)
def test_gol_matrix(golhip, golden_dir, size, turns):
    """TestGol: Operations.Run's FinalTurnComplete alive list for 1..16 threads."""
    board = _golden_board(golden_dir, size)
    expected, gold = _golden_alive(golden_dir, size, turns)
    ops = golhip.Operations(device=0)
    for threads in range(1, 17):
        res = ops.Run(golhip.Request(World=board, Turns=turns, ImageHeight=size, ImageWidth=size,
                                     Threads=threads))
        assert res.TurnsCompleted == turns
        cells = [(c.X, c.Y) for c in res.Alive]
        assert set(cells) == expected, f"{size}x{size}x{turns}-{threads}"
        assert cells == sorted(cells, key=lambda c: (c[1], c[0]))  # row-major, broker.go:50-55
        assert np.array_equal(res.World, gold)


@pytest.mark.parametrize("size", SIZES)
def test_gol_matrix_byte_board(golhip, golden_dir, size):
    """TestGol through a broker that keeps the board one byte per cell (layout="bytes": the
    byte pipeline for 100 turns), for every turn count of the matrix."""
    board = _golden_board(golden_dir, size)
    ops = golhip.Operations(device=0, layout="bytes", shards=2, same_device=True)  # (bytes: one GPU)
    for turns in TURNS:
        expected, gold = _golden_alive(golden_dir, size, turns)
        for threads in (1, 5):
            res = ops.Run(golhip.Request(World=board, Turns=turns, ImageHeight=size, ImageWidth=size,
                                         Threads=threads))
            assert res.TurnsCompleted == turns
            assert set((c.X, c.Y) for c in res.Alive) == expected, f"{size}x{size}x{turns}-{threads}"
            assert np.array_equal(res.World, gold)


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("turns", TURNS)
def test_pgm_output(golhip, golden_dir, tmp_path, size, turns):
    """TestPgm: the P5 file written from the device is byte-identical to check/images."""
    with golhip.Engine(size, size, device=0) as e:
        e.load_bytes(_golden_board(golden_dir, size))
        e.step(turns)
        out = tmp_path / f"{size}x{size}x{turns}.pgm"
        e.write_pgm(str(out))
    with open(os.path.join(golden_dir, "check", "images", f"{size}x{size}x{turns}.pgm"), "rb") as f:
        assert out.read_bytes() == f.read()


@pytest.mark.parametrize("size", SIZES)
def test_alive_counts_csv(golhip, golden_dir, size):
    """TestAlive: alive count after every turn 1..10000 equals check/alive/<s>x<s>.csv."""
    expected = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", f"{size}x{size}.csv"))
    with golhip.Engine(size, size, device=0) as e:
        e.load_bytes(_golden_board(golden_dir, size))
        for t in range(1, 10001):
            e.step(1)
            assert e.alive_count() == expected[t], f"turn {t}"


def test_alive_counts_chunked(golhip, golden_dir):
    """The same counts when stepping in k-turn launches of mixed sizes (temporal blocking)."""
    expected = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", "512x512.csv"))
    with golhip.Engine(512, 512, device=0, turns_per_launch=16) as e:
        e.load_bytes(_golden_board(golden_dir, 512))
        t = 0
        for chunk in [1, 2, 3, 5, 8, 13, 16, 16, 31, 100, 250, 555] * 6:
            e.step(chunk)
            t += chunk
            assert e.alive_count() == expected[t], f"turn {t}"


def test_alive_parity_rule(golhip, golden_dir):
    """count_test.go:47-51: after 10000 turns 512x512 alternates 5565 (even) / 5567 (odd)."""
    with golhip.Engine(512, 512, device=0) as e:
        e.load_bytes(_golden_board(golden_dir, 512))
        e.step(10000)
        for t in range(10001, 10011):
            e.step(1)
            assert e.alive_count() == (5565 if t % 2 == 0 else 5567)


# ------------------------------------------------------------------ kernels vs oracle
@pytest.mark.parametrize("shape", [(64, 64), (128, 256), (100, 192), (37, 320), (1, 64), (2, 128), (3, 64),
                                   (256, 64 * 65), (16, 16), (48, 80), (20, 100), (7, 33), (50, 96), (33, 160),
                                   (300, 32 * 45)])
@pytest.mark.parametrize("turns", [1, 2, 7, 33])
def test_random_boards_vs_oracle(golhip, shape, turns):
    H, W = shape
    rng = np.random.default_rng(H * 1000 + W + turns)
    board = (rng.random((H, W)) < 0.35).astype(np.uint8) * 255
    small = H * W * turns < 2_000_000 or W % 64
    ref = O.run(board, turns) if small else O.unpack(O.bits_run(O.pack(board), turns))
    with golhip.Engine(H, W, device=0) as e:
        e.load_bytes(board)
        e.step(turns)
        assert np.array_equal(e.store_bytes(), ref)
        assert e.alive_count() == int(np.count_nonzero(ref))


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("cpl", [32, 64, 128])
def test_kernel_variants_vs_bit_oracle(golhip, k, cpl):
    """Every (turns per launch, cells per lane) instantiation on a random torus."""
    if k == 16 and cpl == 128:
        pytest.skip("k=16 is built for 32/64 cells per lane only")
    H, W = 300, 64 * 70
    words = O.random_words(11 + k, 0, H, W // 64)
    ref = O.bits_run(words, 45)
    with golhip.Engine(H, W, device=0, turns_per_launch=k, cells_per_lane=cpl) as e:
        e.load_random(11 + k)
        assert e.hash() == O.hash_words(words)
        e.step(45)
        assert e.hash() == O.hash_words(ref)
        assert np.array_equal(e.store_bytes(), O.unpack(ref))


@pytest.mark.parametrize("k,cpl", [(1, 128), (2, 128), (4, 128), (8, 128), (12, 128), (1, 64), (4, 64), (8, 64),
                                   (12, 64), (16, 64)])
@pytest.mark.parametrize("shape", [(300, 1024), (97, 2048), (64, 3072), (33, 8192), (5, 1024)])
def test_band_layout_vs_bit_oracle(golhip, k, cpl, shape):
    """Band-layout kernel (bit b of word w = cell b*W/32 + w) for every (k, words per lane):
    W = 1024 makes one wave span the 32-word row several times (column wrap by rotation)."""
    H, W = shape
    seed = 100 + k + W
    words = O.random_words(seed, 0, H, W // 64)
    ref, counts = O.bits_run(words, 45, with_counts=True)
    with golhip.Engine(H, W, device=0, turns_per_launch=k, cells_per_lane=cpl, layout="band") as e:
        e.load_random(seed)
        info = e.info()
        assert info["layout"] == "band" and info["cells_per_lane"] == cpl
        assert info["turns_per_launch"] == min(k, 16 if H >= 16 else 4 if H >= 4 else 1)
        if k == 12:
            assert info["turns_per_launch"] in (12, 4)  # split pipeline (4 waves x 3 turns) / one wave at 64 cpl
        e.step(20)
        assert e.alive_count() == counts[19]  # popcount on the band layout
        e.step(25)
        assert e.hash() == O.hash_words(ref)
        assert np.array_equal(e.store_bytes(), O.unpack(ref))
        e.step(3)  # back to band after a read
        assert e.alive_count() == O.popcount_words(O.bits_run(ref, 3))


def test_band_layout_standard_agree(golhip):
    """layout=band and layout=standard engines agree on a board loaded from bytes, on the alive
    list (row-major), the PGM bytes and the counts."""
    H, W = 200, 4096
    rng = np.random.default_rng(8)
    board = (rng.random((H, W)) < 0.3).astype(np.uint8) * 255
    out = []
    for layout in ("standard", "band"):
        with golhip.Engine(H, W, device=0, layout=layout) as e:
            e.load_bytes(board)
            e.step(29)
            out.append((e.store_bytes(), e.alive_cells(), e.alive_count(), e.info()["layout"]))
    assert out[0][3] == "standard" and out[1][3] == "band"
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2]
    assert np.array_equal(out[1][0], O.unpack(O.bits_run(O.pack(board), 29)))


def test_band_convert_device(golhip):
    """gol_dev_band_convert against the numpy restatement of the layout (padded pitch)."""
    import torch
    from golhip.sharded import HipKernels
    rows, W = 9, 4096
    Wd = W // 32
    words = O.random_words(4, 0, rows, W // 64)
    src = torch.zeros((rows, Wd + 8), dtype=torch.int32, device="cuda")
    src[:, :Wd] = torch.from_numpy(words.view(np.int32)).cuda()
    band = torch.full((rows, Wd + 4), -1, dtype=torch.int32, device="cuda")
    back = torch.zeros_like(src)
    k = HipKernels()
    k.Wd = Wd
    k.band_convert(True, src, band)
    k.band_convert(False, band, back)
    torch.cuda.synchronize()
    assert np.array_equal(band[:, :Wd].cpu().numpy().view(np.uint32), O.to_band(words))
    assert (band[:, Wd:] == -1).all()  # padding untouched
    assert np.array_equal(back[:, :Wd].cpu().numpy().view(np.uint64), words)


@pytest.mark.parametrize("strip", [1, 5, 32, 97])
def test_strip_sizes(golhip, strip):
    H, W = 211, 64 * 9
    words = O.random_words(5, 0, H, W // 64)
    ref = O.bits_run(words, 20)
    with golhip.Engine(H, W, device=0, turns_per_launch=4, strip_rows=strip) as e:
        e.load_random(5)
        e.step(20)
        assert e.hash() == O.hash_words(ref)


def test_non_binary_bytes_first_turn(golhip):
    """worker.go:26-37: only exactly-0 cells are born, only exactly-255 cells count/survive;
    other bytes become 0.  Before turn 1 the loaded bytes are returned unchanged and count
    as alive in the list (broker.go:52 uses != 0)."""
    rng = np.random.default_rng(3)
    for H, W in [(64, 128), (33, 48)]:
        board = rng.choice(np.array([0, 255, 1, 7, 128, 254], dtype=np.uint8), size=(H, W),
                           p=[.45, .4, .05, .04, .03, .03])
        with golhip.Engine(H, W, device=0) as e:
            e.load_bytes(board)
            assert np.array_equal(e.store_bytes(), board)
            assert e.alive_count() == int(np.count_nonzero(board))
            cells = e.alive_cells()
            assert [tuple(c) for c in cells.tolist()] == O.alive_cells(board)
            e.step(1)
            ref1 = O.run(board, 1)
            assert np.array_equal(e.store_bytes(), ref1)
            e.step(9)
            assert np.array_equal(e.store_bytes(), O.run(board, 10))


def test_next_state_slab_vs_oracle(golhip, golden_dir):
    """GameOfLifeOperations.Update over every slab of the broker's partition."""
    board = _golden_board(golden_dir, 512)
    worker = golhip.GameOfLifeOperations()
    for threads in (1, 3, 4, 7, 16):
        slabs = []
        for i in range(threads):
            y0, y1 = golhip.partition_rows(512, threads, i)
            assert (y0, y1) == O.partition(512, threads, i)
            res = worker.Update(golhip.Request(World=board, StartY=y0, EndY=y1, Worker=i))
            assert np.array_equal(res.WorkSlice, O.next_state_slab(board, y0, y1))
            slabs.append(res.WorkSlice)
        assert np.array_equal(np.concatenate(slabs), O.run(board, 1))
    rng = np.random.default_rng(9)
    odd = rng.choice(np.array([0, 255, 3], dtype=np.uint8), size=(50, 70))
    assert np.array_equal(golhip.next_state_slab(odd, 13, 41), O.next_state_slab(odd, 13, 41))


def test_alive_cells_row_major(golhip):
    rng = np.random.default_rng(4)
    board = (rng.random((130, 64 * 5)) < 0.2).astype(np.uint8) * 255
    with golhip.Engine(130, 320, device=0) as e:
        e.load_bytes(board)
        e.step(3)
        ref = O.run(board, 3)
        got = [tuple(c) for c in e.alive_cells().tolist()]
        assert got == O.alive_cells(ref)
        part = e.alive_cells(cap=17)
        assert [tuple(c) for c in part.tolist()] == O.alive_cells(ref)[:17]


def test_empty_and_full_boards(golhip):
    for fill, turns, expect in [(0, 5, 0), (255, 1, 0)]:
        board = np.full((64, 128), fill, dtype=np.uint8)
        with golhip.Engine(64, 128, device=0) as e:
            e.load_bytes(board)
            e.step(turns)
            assert e.alive_count() == expect
            assert len(e.alive_cells()) == expect


def test_glider_translation(golhip):
    """A glider moves (1,1) every 4 turns; on a torus it comes back after 4*H turns."""
    H = W = 64
    board = np.zeros((H, W), dtype=np.uint8)
    for x, y in [(1, 0), (2, 1), (0, 2), (1, 2), (2, 2)]:
        board[y, x] = 255
    with golhip.Engine(H, W, device=0) as e:
        e.load_bytes(board)
        e.step(4)
        assert np.array_equal(e.store_bytes(), np.roll(np.roll(board, 1, 0), 1, 1))
        e.step(4 * H - 4)
        assert np.array_equal(e.store_bytes(), board)


def test_errors_are_codes_not_crashes(golhip):
    with pytest.raises(golhip.GolError):
        golhip.Engine(0, 64)
    with golhip.Engine(32, 64, device=0) as e:
        with pytest.raises(golhip.GolError):
            e.step(-1)
    with golhip.Engine(32, 48, device=0) as e:
        with pytest.raises(golhip.GolError):
            e.load_random(1)  # needs W % 64 == 0
    ops = golhip.Operations(device=0)
    with pytest.raises(golhip.GolError):
        ops.RetrieveCurrentData(golhip.Request(ImageHeight=16, ImageWidth=16))  # no Run yet
    with pytest.raises(golhip.GolError):
        ops.Run(golhip.Request(World=np.zeros((16, 16), np.uint8), Turns=1, ImageHeight=16, ImageWidth=16,
                               Threads=0))


# ------------------------------------------------------------------ full-size properties
def test_tiled_board_matches_small_torus(golhip):
    """A torus tiled with copies of a small torus evolves as the small one (every tile equal to
    the oracle's small-board result) -- checks the kernel at a size the oracle cannot run."""
    th, tw, reps_y, reps_x, turns = 256, 512, 64, 128, 40
    rng = np.random.default_rng(21)
    tile = (rng.random((th, tw)) < 0.4).astype(np.uint8) * 255
    ref = O.unpack(O.bits_run(O.pack(tile), turns))
    big = np.tile(tile, (reps_y, reps_x))  # 16384 x 65536
    with golhip.Engine(th * reps_y, tw * reps_x, device=0) as e:
        e.load_bytes(big)
        del big
        e.step(turns)
        got = e.store_bytes().reshape(reps_y, th, reps_x, tw)
        assert (got == ref[None, :, None, :]).all()
        assert e.alive_count() == reps_y * reps_x * int(np.count_nonzero(ref))


def test_bench_size_k_and_layout_invariance(golhip):
    """2^17 x 2^20 (the bench's per-GPU torus) through the engine: k=1, 8 and 16 launches on the
    standard layout and k=1, 8 and 12 on the band layout give the same board hash, and the count
    fused into the last launch equals the popcount kernel."""
    import torch
    H, W, turns = 1 << 17, 1 << 20, 48
    hashes = []
    for layout, k in (("standard", 1), ("standard", 8), ("standard", 16), ("band", 1), ("band", 8), ("band", 12)):
        with golhip.Engine(H, W, device=0, layout=layout, turns_per_launch=k) as e:
            assert e.info()["layout"] == layout and e.info()["turns_per_launch"] == k
            e.load_random(1)
            fused = e.step_counted(turns, turns).tolist()
            assert fused == [e.alive_count()]
            hashes.append(e.hash())
        torch.cuda.empty_cache()
    assert len(set(hashes)) == 1


# ------------------------------------------------------------------ broker control path
def test_alive_events_during_run_pause_quit(golhip, golden_dir):
    """count_test.go:17-69 (TestAlive) through the broker mirror: a 10^8-turn Run on 512x512
    with 8 threads; RetrieveCurrentData (the 2-s ticker of distributor.go:39-51) must return
    (turn, count) pairs that match check/alive (or the 5565/5567 parity rule past turn 10000);
    Pause freezes the turn (broker.go:251-254), a second Pause resumes, Quit ends the Run with
    the turns completed so far (broker.go:236-239)."""
    import threading
    import time
    expected = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", "512x512.csv"))
    board = _golden_board(golden_dir, 512)
    ops = golhip.Operations(device=0)
    req = golhip.Request(World=board, Turns=10**8, ImageHeight=512, ImageWidth=512, Threads=8)
    out = {}
    th = threading.Thread(target=lambda: out.update(res=ops.Run(req)))
    th.start()
    try:
        seen = []
        deadline = time.time() + 60
        while len(seen) < 5 and time.time() < deadline:
            time.sleep(0.05)
            r = ops.RetrieveCurrentData(golhip.Request(ImageHeight=512, ImageWidth=512), alive=False, world=False)
            t, c = r.TurnsCompleted, r.AliveCount
            if t == 0:
                assert c == 0  # cWorld is all-zero before the first turn (broker.go:67-70)
                continue
            want = expected[t] if t <= 10000 else (5565 if t % 2 == 0 else 5567)
            assert c == want, f"turn {t}: {c} != {want}"
            seen.append(t)
        assert len(seen) == 5 and seen == sorted(seen)
        ops.Pause()
        time.sleep(0.2)
        assert ops.paused
        t1 = ops.RetrieveCurrentData(golhip.Request(ImageHeight=512, ImageWidth=512), alive=False).TurnsCompleted
        time.sleep(0.2)
        r2 = ops.RetrieveCurrentData(golhip.Request(ImageHeight=512, ImageWidth=512))
        assert r2.TurnsCompleted == t1  # paused: no progress
        assert len(r2.Alive) == r2.AliveCount
        ops.Pause()  # resume
        time.sleep(0.2)
        assert not ops.paused
        assert ops.RetrieveCurrentData(golhip.Request(ImageHeight=512, ImageWidth=512),
                                       alive=False, world=False).TurnsCompleted > t1
    finally:
        ops.Quit()
        th.join(60)
    assert not th.is_alive()
    res = out["res"]
    t = res.TurnsCompleted
    assert 0 < t < 10**8
    want = expected[t] if t <= 10000 else (5565 if t % 2 == 0 else 5567)
    assert len(res.Alive) == want
    ys, xs = np.nonzero(res.World)
    assert [(c.X, c.Y) for c in res.Alive] == list(zip(xs.tolist(), ys.tolist()))
    ops.SuperQuit()
    with pytest.raises(golhip.GolError):
        ops.Run(golhip.Request(World=board, Turns=1, ImageHeight=512, ImageWidth=512, Threads=1))


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32])
def test_byte_board_k_turn_kernel(golhip, k):
    """gol_dev_bytes_step_k (0/255 byte board, k turns per launch) against the oracle, with the
    torus wrap through top/bot and a split into two launches (row ranges)."""
    import torch
    from golhip._lib import check, lib
    H, W, turns = 203, 32 * 67, 3 * k
    rng = np.random.default_rng(100 + k)
    board = (rng.random((H, W)) < 0.4).astype(np.uint8) * 255
    ref = O.run(board, turns) if H * W * turns < 3_000_000 else None
    a = torch.from_numpy(board).cuda()
    b = torch.empty_like(a)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(turns // k):
        top = a[H - k:]
        check(lib().gol_dev_bytes_step_k(top.data_ptr(), a.data_ptr(), a.data_ptr(), b.data_ptr(), H, W, W,
                                         0, 100, k, 0, None, st))
        check(lib().gol_dev_bytes_step_k(top.data_ptr(), a.data_ptr(), a.data_ptr(), b.data_ptr(), H, W, W,
                                         100, H - 100, k, 0, None, st))
        a, b = b, a
    got = a.cpu().numpy()
    if ref is None:
        ref = O.run(board, turns)
    assert np.array_equal(got, ref)


def _bytes_k_steps(board, k, launches, strip, splits):
    """gol_dev_bytes_step_k on a (H, W) 0/255 torus: `launches` k-turn launches, each over the row
    ranges `splits` (several launches per turn step); returns the board after k*launches turns."""
    import torch
    from golhip._lib import check, lib
    H, W = board.shape
    a = torch.from_numpy(board).cuda()
    b = torch.empty_like(a)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(launches):
        top = a[H - k:]
        for r0, r1 in splits:
            check(lib().gol_dev_bytes_step_k(top.data_ptr(), a.data_ptr(), a.data_ptr(), b.data_ptr(), H, W, W,
                                             r0, r1 - r0, k, strip, None, st))
        a, b = b, a
    torch.cuda.synchronize()
    flags = ctypes.c_uint32()
    check(lib().gol_dev_error(-1, ctypes.byref(flags)))
    return a.cpu().numpy()


@pytest.mark.parametrize("H,strip", [(620, 130), (1100, 0), (700, 64)])
def test_byte_pipe_several_strips(golhip, H, strip):
    """The k = 32 byte pipeline (8 waves x 4 turns) with several strips per launch (blockIdx.y > 0):
    explicit 130- and 64-row strips and the automatic round-tiled strip at >= 1024 rows, against
    the bit oracle; the second launch splits the rows in two ranges (strip edges inside a launch)."""
    W = 32 * 96
    rng = np.random.default_rng(H + strip)
    board = (rng.random((H, W)) < 0.4).astype(np.uint8) * 255
    got = _bytes_k_steps(board, 32, 2, strip, [(0, H)])
    ref = O.unpack(O.bits_run(O.pack(board), 64))
    assert np.array_equal(got, ref)
    got2 = _bytes_k_steps(board, 32, 1, strip, [(0, 333), (333, H)])
    assert np.array_equal(got2, O.unpack(O.bits_run(O.pack(board), 32)))


def test_byte_pipe_paired_narrow_board(golhip):
    """Two column groups and enough rows for the one-round rank split with a paired range per
    CU (two workgroups walking one range from both ends, meeting wherever the faster one got to)
    plus a lone rank: 32768 x 2112 bytes, two k = 32 launches against the bit oracle."""
    H, W = 32768, 32 * 66
    words = O.random_words(5, 0, H, W // 64)
    board = O.unpack(words)
    got = _bytes_k_steps(board, 32, 2, 0, [(0, H)])
    assert O.hash_words(O.pack(got)) == O.hash_words(O.bits_run(words, 64))


def test_byte_board_engine_counted_paired(golhip):
    """A width that is a multiple of 32 but not of 64 keeps the engine on the 0/255 byte board:
    with k = 32 its launches take the byte pipeline's one-round rank split (paired ranges); the
    alive count of every launch (fused) and the board against the literal port (16 threads)."""
    H, W = 28672, 32 * 65
    rng = np.random.default_rng(2080)
    board = (rng.random((H, W)) < 0.35).astype(np.uint8) * 255
    with golhip.Engine(H, W, device=0, turns_per_launch=32) as e:
        e.load_bytes(board)
        counts = e.step_counted(64, 32)
        got = e.store_bytes()
    mid = O.run(board, 32, 16)
    ref = O.run(mid, 32, 16)
    assert counts.tolist() == [int(np.count_nonzero(mid)), int(np.count_nonzero(ref))]
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("shape", [(32, 64), (50, 128), (203, 2048), (1000, 4096), (4096, 32 * 97 * 2)])
def test_bytes_layout_engine(golhip, shape):
    """GOL_LAYOUT_BYTES keeps a W % 64 == 0 board as the reference's bytes (config 2's path through
    the engine): load_random gives the bit boards' cells as 0/255, k = 32 launches take the byte
    pipeline with the fused count, a short tail takes the blocked byte kernel; bit-board calls
    are EINVAL."""
    H, W = shape
    words = O.random_words(7, 0, H, W // 64)
    with golhip.Engine(H, W, device=0, layout="bytes") as e:
        info = e.info()
        assert info["layout"] == "bytes" and info["turns_per_launch"] == 32 and not info["bit_mode"]
        e.load_random(7)
        assert np.array_equal(e.store_bytes(), O.unpack(words))
        counts = e.step_counted(64, 32)
        e.step(5)
        ref, rc = O.bits_run(words, 69, with_counts=True)
        assert counts.tolist() == [rc[31], rc[63]]
        assert np.array_equal(e.store_bytes(), O.unpack(ref))
        assert e.alive_count() == rc[68] and e.turn == 69
        with pytest.raises(golhip.GolError):
            e.hash()


def test_byte16k_engine_full_size(golhip):
    """Config 2's engine path at its size: Engine(16384, 16384, layout="bytes"),
    load_random(1), two counted k = 32 launches of the byte pipeline -- the path bench.py's byte16k
    line times -- against the bit oracle's 64 turns: the board and both fused counts."""
    H = W = 16384
    with golhip.Engine(H, W, device=0, layout="bytes") as e:
        assert e.info()["turns_per_launch"] == 32 and e.info()["layout"] == "bytes"
        e.load_random(1)
        counts = e.step_counted(64, 32)
        got = e.store_bytes()
    ref, rc = O.bits_run(O.random_words(1, 0, H, W // 64), 64, with_counts=True)
    assert counts.tolist() == [int(rc[31]), int(rc[63])]
    assert np.array_equal(got, O.unpack(ref))


def test_default_k_on_w32_byte_board(golhip):
    """a board of W % 64 == 32 is a byte board whatever the layout, and its default k
    is the byte pipeline's 32 (round 5 changed it from 8): 203 x 32*67 at the default k -- two
    counted k = 32 launches and a 5-turn tail of the blocked kernel -- against the literal port;
    the info call reports what the next launch runs (1 before the exact first turn of non-0/255
    bytes)."""
    H, W = 203, 32 * 67
    rng = np.random.default_rng(67)
    board = (rng.random((H, W)) < 0.4).astype(np.uint8) * 255
    with golhip.Engine(H, W, device=0) as e:
        assert e.info()["layout"] == "bytes" and e.info()["turns_per_launch"] == 32
        e.load_bytes(board)
        counts = e.step_counted(64, 32)
        e.step(5)
        got = e.store_bytes()
        odd = board.copy()
        odd[0, 0] = 7
        e.load_bytes(odd)
        assert e.info()["turns_per_launch"] == 1
    mid = O.run(board, 32, 4)
    end = O.run(mid, 32, 4)
    assert counts.tolist() == [int(np.count_nonzero(mid)), int(np.count_nonzero(end))]
    assert np.array_equal(got, O.run(end, 5, 4))


def test_bytes_layout_timing_and_rank_refusal(golhip):
    """The byte board's launches are timed like the bit board's (bench.py byte16k reads them), and
    a byte board does not shard."""
    H, W = 512, 1024
    with golhip.Engine(H, W, device=0, layout="bytes") as e:
        e.load_random(3)
        e.set_timing(True)
        e.step_counted(96, 32)
        t = e.timing()
        e.set_timing(False)
        assert t["launches"] == 3 and t["mean_cell_updates"] == H * W * 32 and t["mean_ms"] > 0
    with pytest.raises(golhip.GolError):
        golhip.Engine(H, W, device=0, layout="bytes", shards=2, same_device=True)


def test_band_paired_narrow_board(golhip):
    """One band column group (W = 2048) over 65536 rows: the one-round rank split gives every CU
    256 rows in two paired ranges of ~128 rows (4K = 48 rows of fill each); 25 turns (two k = 12
    launches and a 1-turn one) against the bit oracle."""
    H, W = 65536, 2048
    with golhip.Engine(H, W, device=0) as e:
        assert e.info()["layout"] == "band" and e.info()["turns_per_launch"] == 12
        e.load_random(11)
        counts = e.step_counted(24, 12)
        e.step(1)
        ref, rc = O.bits_run(O.random_words(11, 0, H, W // 64), 25, with_counts=True)
        assert counts.tolist() == [rc[11], rc[23]]
        assert e.hash() == O.hash_words(ref)


def test_byte16k_full_size_parity(golhip):
    """Config 2 at its size: the 16384 x 16384 byte board, two k = 32 launches (the bench's
    kernel, automatic strips: many strips per column group) against the bit oracle's 64 turns."""
    H = W = 16384
    words = O.random_words(1, 0, H, W // 64)
    board = O.unpack(words)
    got = _bytes_k_steps(board, 32, 2, 0, [(0, H)])
    ref = O.bits_run(words, 64)
    assert O.hash_words(O.pack(got)) == O.hash_words(ref)
    assert np.array_equal(got, O.unpack(ref))


# ------------------------------------------------------------------ CellFlipped stream
def _check_flips(e, board, turns):
    """step_flips() per turn == oracle diff of consecutive generations; replaying the flips
    onto the previous board gives the new one (what an SDL view does, sdl/loop.go:9-53)."""
    prev = board
    shown = (board != 0).astype(np.uint8)
    for t in range(1, turns + 1):
        got = [tuple(c) for c in e.step_flips().tolist()]
        cur = O.run(board, t)
        assert got == O.flipped_cells(prev, cur), f"turn {t}"
        for x, y in got:
            shown[y, x] ^= 1
        assert np.array_equal(shown, (cur != 0).astype(np.uint8))
        assert e.turn == t
        prev = cur
    assert np.array_equal(e.store_bytes(), prev)


def test_step_flips_golden_board(golhip, golden_dir):
    board = _golden_board(golden_dir, 64)
    with golhip.Engine(64, 64, device=0) as e:
        e.load_bytes(board)
        _check_flips(e, board, 12)


@pytest.mark.parametrize("shape", [(130, 1024), (33, 48), (40, 96)])
def test_step_flips_layouts(golhip, shape):
    """Band-capable width (after k-turn band steps), a byte-only width and a standard one."""
    H, W = shape
    rng = np.random.default_rng(H + W)
    board = (rng.random((H, W)) < 0.35).astype(np.uint8) * 255
    with golhip.Engine(H, W, device=0) as e:
        e.load_bytes(board)
        e.step(12)
        start = O.run(board, 12)
        prev = start
        for t in range(1, 4):
            got = [tuple(c) for c in e.step_flips().tolist()]
            cur = O.run(start, t)
            assert got == O.flipped_cells(prev, cur)
            prev = cur
        assert e.turn == 15
        part = e.step_flips(cap=5)
        assert [tuple(c) for c in part.tolist()] == O.flipped_cells(prev, O.run(start, 4))[:5]


def test_step_flips_non_binary_first_turn(golhip):
    """Turn 1 from bytes other than 0/255: a non-zero byte that dies is a flip (alive = != 0)."""
    rng = np.random.default_rng(11)
    for H, W in [(64, 128), (33, 48)]:
        board = rng.choice(np.array([0, 255, 1, 7, 128], dtype=np.uint8), size=(H, W), p=[.5, .35, .05, .05, .05])
        with golhip.Engine(H, W, device=0) as e:
            e.load_bytes(board)
            _check_flips(e, board, 3)
