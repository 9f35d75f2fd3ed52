"""The pipelines' fill-block skip, checked on a CPU model of the row pipeline (no GPU).

band_pipe_kernel (gol_kernels.hip, `run`: the fill-trip loop) and bytes_pipe_kernel (`nskip`)
stream the rows of a strip through K stages, one generation each; stage g at stream step t
holds its last three input rows and emits the next state of the middle one, so the last stage
emits row t - K at generation K, valid from step 2K on (the rows stored).  (Since round 5 the
stages take their rows in pairs -- a block is one or two pair steps -- which computes the same
function of the stream: one row of delay per stage.)  A wave whose first stage is g0 leaves its
stages' state untouched and passes the rows on unchanged for the blocks of RPB steps that end
before step 2 g0.  The model below executes exactly that and compares every stored row with the
oracle's K-turn evolution of the torus (oracle.np_next_state, the numpy restatement of
worker.go:15-70); skipping one block more must break it."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def _life(a, m, c):
    """next state of row m (bool) from the rows above / below, torus along the row"""
    n = np.zeros(m.shape, dtype=np.int8)
    for i, r in enumerate((a, m, c)):
        for dx in (-1, 0, 1):
            if i != 1 or dx:
                n += np.roll(r, dx).astype(np.int8)
    return (n == 3) | (m & (n == 2))


def _pipeline(rows, K, KW, skip_blocks, rpb=3):
    """rows: the stream (bool rows); skip_blocks(wv) = blocks b (of rpb rows) whose rule wave wv
    skips"""
    zero = np.zeros_like(rows[0])
    state = [[zero, zero, zero] for _ in range(K)]
    out = []
    for t, r in enumerate(rows):
        cur = r
        for g in range(K):
            if t // rpb < skip_blocks(g // KW):
                continue  # fill block: passed on unchanged, state untouched
            st = state[g]
            st.pop(0)
            st.append(cur)
            cur = _life(*st)
        out.append(cur)
    return out


def _band_skip(KW):  # band_pipe_kernel: blocks of 2 rows, whole loop trips of NS = 4 blocks below g0
    return lambda wv: 4 * ((KW * wv) // 4)


def _bytes_skip(KW):  # bytes_pipe_kernel: blocks of 4 rows, every block that ends before 2 g0
    return lambda wv: (2 * KW * wv) // 4


def _bytes_skip_r4(KW):  # round 4's byte pipeline: blocks of 3 rows, skip_b = 2 g0 / 3
    return lambda wv: (2 * KW * wv) // 3


@pytest.mark.parametrize("K,KW,mk,rpb", [(12, 3, _band_skip, 2), (16, 4, _band_skip, 2), (32, 4, _bytes_skip, 4),
                                         (12, 3, _bytes_skip, 4), (32, 4, _bytes_skip_r4, 3)])
@pytest.mark.parametrize("seed", [1, 2])
def test_fill_skip_keeps_every_stored_row(K, KW, mk, rpb, seed):
    H, W, s0, s1 = 96, 40, 7, 61
    rng = np.random.default_rng(seed)
    board = np.where(rng.random((H, W)) < 0.4, 255, 0).astype(np.uint8)
    ref = board
    for _ in range(K):
        ref = O.np_next_state(ref)
    rows = [board[(s0 - K + t) % H] == 255 for t in range(s1 - s0 + 2 * K)]
    out = _pipeline(rows, K, KW, mk(KW), rpb)
    for t in range(2 * K, len(rows)):
        assert np.array_equal(out[t], ref[s0 + t - 2 * K] == 255), (t, s0 + t - 2 * K)
    # and the skip is what the kernels save: nothing for the first wave, more downstream
    assert mk(KW)(0) == 0 and mk(KW)(K // KW - 1) > 0


@pytest.mark.parametrize("K,KW,rpb", [(12, 3, 2), (32, 4, 4), (32, 4, 3)])
def test_one_block_more_breaks_it(K, KW, rpb):
    H, W, s0, s1 = 96, 40, 7, 61
    rng = np.random.default_rng(3)
    board = np.where(rng.random((H, W)) < 0.4, 255, 0).astype(np.uint8)
    ref = board
    for _ in range(K):
        ref = O.np_next_state(ref)
    rows = [board[(s0 - K + t) % H] == 255 for t in range(s1 - s0 + 2 * K)]
    P = K // KW
    over = lambda wv: (2 * KW * wv) // rpb + (1 if wv == P - 1 else 0)  # noqa: E731
    out = _pipeline(rows, K, KW, over, rpb)
    assert any(not np.array_equal(out[t], ref[s0 + t - 2 * K] == 255) for t in range(2 * K, len(rows)))
