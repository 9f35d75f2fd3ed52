"""Pin the CPU oracle against the reference's own golden fixtures.

Fixtures are byte copies of /root/reference/check/{images,alive} and
/root/reference/images (tests/golden/SHA256SUMS).  These are the vectors the
reference's end-to-end tests use: gol_test.go:15-47 (alive sets from
check/images), pgm_test.go:10-42 (PGM bytes), count_test.go:17-69 (alive
counts per turn from check/alive, parity rule after turn 10000).
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import oracle as O

SIZES = [16, 64, 512]
TURNS = [0, 1, 100]


def test_fixture_checksums(golden_dir):
    with open(os.path.join(golden_dir, "SHA256SUMS")) as f:
        for line in f:
            digest, name = line.split()
            with open(os.path.join(golden_dir, name), "rb") as g:
                assert hashlib.sha256(g.read()).hexdigest() == digest, name


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("turns", TURNS)
def test_oracle_pgm_golden(golden_dir, size, turns):
    """Literal worker.go port + broker turn loop reproduces check/images byte-for-byte
    (header included: gol/io.go:52-59)."""
    W, H, board = O.read_pgm(os.path.join(golden_dir, "images", f"{size}x{size}.pgm"), size, size)
    out = O.run(board, turns, threads=1)
    path = os.path.join(golden_dir, "check", "images", f"{size}x{size}x{turns}.pgm")
    with open(path, "rb") as f:
        assert O.pgm_bytes(out) == f.read()


@pytest.mark.parametrize("threads", [1, 2, 3, 4, 7, 16])
def test_oracle_threads_do_not_change_result(golden_dir, threads):
    """broker.go:135-206: Threads only changes the slab split, never the board."""
    _, _, board = O.read_pgm(os.path.join(golden_dir, "images", "64x64.pgm"))
    ref = O.run(board, 10, threads=1)
    assert np.array_equal(O.run(board, 10, threads=threads), ref)


@pytest.mark.parametrize("size", SIZES)
def test_oracle_alive_csv(golden_dir, size):
    """check/alive/<s>x<s>.csv: alive count after each of turns 1..10000."""
    _, _, board = O.read_pgm(os.path.join(golden_dir, "images", f"{size}x{size}.pgm"))
    expected = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", f"{size}x{size}.csv"))
    assert sorted(expected) == list(range(1, 10001))
    if size % 64 == 0:
        _, counts = O.bits_run(O.pack(board), 10000, with_counts=True)
        got = {t + 1: int(c) for t, c in enumerate(counts)}
    else:
        got = {}
        w = board
        for t in range(1, 10001):
            w = O.np_next_state(w)
            got[t] = int(np.count_nonzero(w))
    assert got == expected


def test_oracle_alive_parity_rule(golden_dir):
    """count_test.go:47-51: after turn 10000 the 512x512 count alternates 5565 (even) / 5567 (odd)."""
    _, _, board = O.read_pgm(os.path.join(golden_dir, "images", "512x512.pgm"))
    _, counts = O.bits_run(O.pack(board), 10006, with_counts=True)
    for t in range(10001, 10007):
        assert counts[t - 1] == (5565 if t % 2 == 0 else 5567)


@pytest.mark.parametrize("size", SIZES)
def test_oracle_alive_cells_golden(golden_dir, size):
    """gol_test.go:88-129 readAliveCells treats any nonzero byte as alive; broker.go:47-58."""
    _, _, board = O.read_pgm(os.path.join(golden_dir, "images", f"{size}x{size}.pgm"))
    out = O.run(board, 1)
    _, _, gold = O.read_pgm(os.path.join(golden_dir, "check", "images", f"{size}x{size}x1.pgm"))
    cells = O.alive_cells(out)
    ys, xs = np.nonzero(gold)
    assert cells == list(zip(xs.tolist(), ys.tolist()))


def test_literal_port_matches_numpy_and_bits_on_random_boards():
    rng = np.random.default_rng(1234)
    for H, W in [(64, 64), (128, 64), (64, 192), (3, 64)]:
        board = (rng.random((H, W)) < 0.4).astype(np.uint8) * 255
        lit = O.run(board, 5, threads=3)
        nump = board
        for _ in range(5):
            nump = O.np_next_state(nump)
        bits = O.unpack(O.bits_run(O.pack(board), 5))
        assert np.array_equal(lit, nump)
        assert np.array_equal(lit, bits)


def test_literal_port_non_binary_bytes():
    """worker.go:26-37: birth needs exactly 0, survival and counting exactly 255;
    any other byte becomes 0 and is never counted."""
    rng = np.random.default_rng(7)
    board = rng.choice(np.array([0, 255, 1, 128, 254], dtype=np.uint8), size=(32, 48), p=[.4, .4, .1, .05, .05])
    assert np.array_equal(O.run(board, 1), O.np_next_state(board))
    assert np.array_equal(O.next_state_slab(board, 5, 17), O.np_next_state(board)[5:17])


@pytest.mark.parametrize("H,T", [(512, 4), (16, 3), (64, 7), (10, 16), (512, 16), (17, 5)])
def test_partition_formula(H, T):
    """broker.go:135-139 even split, 172-206: first H%T slabs get one extra row."""
    spans = [O.partition(H, T, i) for i in range(T)]
    assert spans[0][0] == 0 and spans[-1][1] == H
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0
    sizes = [b - a for a, b in spans]
    rem = H % T
    assert sizes == [H // T + 1] * rem + [H // T] * (T - rem)


def test_random_words_and_hash_are_shardable():
    full = O.random_words(3, 0, 40, 4)
    assert np.array_equal(O.random_words(3, 10, 30, 4), full[10:])
    assert (O.hash_words(full[:10], 0) + O.hash_words(full[10:], 10)) % 2**64 == O.hash_words(full, 0)
    # Bernoulli(1/2) per cell
    assert abs(O.popcount_words(full) / (40 * 4 * 64) - 0.5) < 0.02
