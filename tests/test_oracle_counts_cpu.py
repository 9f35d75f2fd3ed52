"""The multi-threaded oracle (oracle/gol_oracle_mt.c) and the count series it pins.

tests/golden/bench_counts.json -- the series every bench line's counts are checked against
(`config.parity`) -- comes from one GPU stepping each whole torus.  tests/golden/oracle_counts.json
holds the same series computed by the CPU oracle (tools/pin_counts_oracle.py).  Here:
  * the multi-threaded in-place oracle equals the single-threaded oracle (gol_oracle.c) on every
    shape class and thread count, and reproduces the reference's check/alive counts;
  * each stored oracle series is reproducible from the oracle's code (a prefix recomputed);
  * the GPU series equals the oracle's at every point both hold -- BASELINE config 2 (16384^2)
    and config 3 (65536^2) beyond their 10,000 turns, and prefixes of the bench's weak and
    262144^2 boards.
(tests/test_gpu_configs.py `test_oracle_count_series` steps the boards on the GPU to the oracle's
last turn and compares every count and the final board hash.)
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("H,Ww", [(1, 1), (2, 1), (3, 1), (1, 3), (2, 2), (3, 5), (7, 2), (16, 4), (33, 5),
                                  (64, 2), (9, 17), (130, 3)])
def test_mt_oracle_matches_oracle(H, Ww):
    """Every turn's board and count, 1-9 threads (more threads than rows included)."""
    rng = np.random.default_rng(H * 1000 + Ww)
    w = rng.integers(0, 2**64, size=(H, Ww), dtype=np.uint64)
    ref, rc = O.bits_run(w, 24, with_counts=True)
    for T in (1, 2, 3, 8, 9):
        x = w.copy()
        assert O.mt_bits_run(x, 24, 1, T).tolist() == rc.tolist(), T
        assert np.array_equal(x, ref), T
        x = w.copy()
        assert O.mt_bits_run(x, 24, 6, T).tolist() == rc[5::6].tolist(), T
        assert np.array_equal(x, ref), T


def test_mt_random_and_hash():
    for H, Ww in [(1, 1), (5, 3), (64, 16)]:
        w = O.mt_random_words(7, H, Ww, 3)
        assert np.array_equal(w, O.random_words(7, 0, H, Ww))
        assert O.mt_hash_words(w, 3) == O.hash_words(w)


def test_mt_oracle_alive_csv(golden_dir):
    """The reference's check/alive/512x512.csv (count_test.go:17-69), turns 1..10000."""
    _, _, board = O.read_pgm(os.path.join(golden_dir, "images", "512x512.pgm"))
    expected = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", "512x512.csv"))
    w = np.ascontiguousarray(O.pack(board))
    counts = O.mt_bits_run(w, 10000, 1, 4)
    assert {t + 1: int(c) for t, c in enumerate(counts)} == expected


@pytest.fixture(scope="module")
def oracle_counts():
    return _load("oracle_counts.json")


def test_oracle_series_reproducible(oracle_counts):
    """The first points of every stored oracle series of a board of <= 2^32 cells, recomputed."""
    n = 0
    for key, rec in oracle_counts["boards"].items():
        H, W, every = rec["H"], rec["W"], rec["every"]
        if H * W > 1 << 32:
            continue
        w = O.mt_random_words(1, H, W // 64, 8)
        pts = min(len(rec["counts"]), 2)
        assert O.mt_bits_run(w, pts * every, every, 8).tolist() == rec["counts"][:pts], key
        n += 1
    assert n >= 3


def test_bench_series_pinned_to_oracle(oracle_counts):
    """Every point of the GPU series (bench_counts.json) that the oracle holds is the oracle's; the
    oracle covers BASELINE config 2 (16384^2) and config 3 (65536^2) past their 10,000 turns, and the
    bench's weak board at N = 1 and 2 and the 262144^2 board past the driver's run (78 counts, 936
    turns)."""
    bench = _load("bench_counts.json")["boards"]
    covered = {}
    for key, rec in oracle_counts["boards"].items():
        assert key in bench, key
        b = bench[key]
        assert (b["H"], b["W"], b["every"]) == (rec["H"], rec["W"], rec["every"]), key
        n = len(rec["counts"])
        assert rec["turns"] == n * rec["every"]
        assert b["counts"][:n] == rec["counts"], key
        covered[key] = rec["turns"]
    assert covered.get("16384x16384", 0) >= 10000
    assert covered.get("65536x65536", 0) >= 10000
    assert covered.get("131072x1048576", 0) >= 936
    assert covered.get("262144x1048576", 0) >= 936  # the weak board at N = 2 (the driver's SCALE run)
    assert covered.get("262144x262144", 0) >= 936
    assert covered.get("4096x65536", 0) >= 600
