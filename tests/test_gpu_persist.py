"""The persistent multi-round band launch (gol_kernels.hip band_persist_pipe_kernel)
against the oracle and against one launch per step.

A one-shard band board (W % 1024 == 0, W >= 8192) steps many k = 12 turns in one launch: tiles
of (strip, column group) claimed round by round, each waiting for its 3 x 3 neighbourhood of the
previous round, rows wrapping inside the shard.  The cases cover
  * boards of a few tiles per round (3 strips x 2 groups: most claims wait for their own
    neighbourhood -- the padding-trip hand-over) up to boards of thousands of tiles,
  * explicit strips down to k rows, uneven last strips and a narrow last column group,
  * counts every 12 / 24 / 36 turns and turn counts that leave a remainder for the per-launch path,
  * chunking: more rounds than one launch takes (GOL_PERSIST_MAX_ROUNDS),
all bit-exact against oracle.bits_run (the oracle's word-parallel restatement, itself pinned to
the literal port of worker.go:15-70 in tests/test_oracle.py) or, at sizes the oracle cannot
run, against the same engine with GOL_STEP_PERSIST.
"""
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


def _run(G, H, W, words, turns, every, **kw):
    e = G.Engine(H, W, persist=True, **kw)
    try:
        e.load_words(0, words)
        counts = e.step_counted(turns, every) if every else e.step(turns)
        out = e.store_words(0, H)
        return out, (None if counts is None else [int(c) for c in counts]), e.turn
    finally:
        e.close()


@pytest.mark.parametrize("H,W,strip,turns,every", [
    (36, 8192, 12, 12 * 6, 12),     # 3 strips x 2 groups (the last 24 words wide): waits on own tiles
    (36, 8192, 0, 12 * 5, 12),      # one strip: every neighbour is the tile itself
    (37, 8192, 12, 12 * 5, 12),     # strips 12, 12, 13 (the last takes the remainder)
    (100, 9216, 0, 12 * 4, 24),     # Wd 288: 2 groups, the last 56 words
    (512, 8192, 37, 12 * 9 + 5, 12),  # a 5-turn remainder on the per-launch path
    (1000, 16384, 96, 12 * 13, 36),
    (256, 32768, 0, 12 * 3, 12),
])
def test_persist_vs_oracle(G, H, W, strip, turns, every):
    words = O.random_words(11 + H, 0, H, W // 64)
    ref, counts = O.bits_run(words, turns, with_counts=True)
    want = [int(c) for c in counts[every - 1::every]]
    out, got, turn = _run(G, H, W, words, turns, every, strip_rows=strip)
    assert turn == turns
    assert got == want
    assert np.array_equal(out, ref)


def test_persist_chunked_rounds(G):
    # 150 rounds: three launches of <= 64 rounds, counts across the chunk boundaries
    H, W = 48, 8192
    words = O.random_words(5, 0, H, W // 64)
    ref, counts = O.bits_run(words, 12 * 150, with_counts=True)
    out, got, _ = _run(G, H, W, words, 12 * 150, 12)
    assert got == [int(c) for c in counts[11::12]]
    assert np.array_equal(out, ref)


def test_persist_step_without_counts(G):
    H, W = 300, 8192
    words = O.random_words(9, 0, H, W // 64)
    ref = O.bits_run(words, 12 * 7 + 3)
    out, _, turn = _run(G, H, W, words, 12 * 7 + 3, 0)
    assert turn == 12 * 7 + 3
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("H,W,strip", [(2048, 65536, 0), (4096, 1 << 20, 0), (8192, 65536, 100)])
def test_persist_matches_per_launch(G, H, W, strip):
    """Boards the oracle is slow on: the persistent launch against one launch per step."""
    res = []
    for persist in (True, False):
        e = G.Engine(H, W, strip_rows=strip, persist=persist)
        try:
            e.load_random(3)
            c = [int(x) for x in e.step_counted(12 * 20, 12)]
            c += [int(x) for x in e.step_counted(12 * 6, 36)]
            res.append((c, e.hash(), e.alive_count()))
        finally:
            e.close()
    assert res[0] == res[1]
    assert res[0][0][-1] == res[0][2]
