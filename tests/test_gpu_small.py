"""Small boards under the latency rule: boards too small to fill the GPU with
strips of max(32, 8k) rows (standard layout) or with 256 tiles of 8k rows (band pipeline) are cut
into ~512 strips of 1-2 rows.  Each case runs the automatic strip against the oracle's
word-parallel restatement (pinned to worker.go:15-70 in tests/test_oracle.py) with a count every
12 turns (so the steps are k-turn launches): 1- and 2-row strips, strips that do not divide the
rows, boards a few strips tall and turn counts with remainders all meet the oracle bit for bit."""
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


@pytest.mark.parametrize("H,W,turns", [
    (512, 512, 37),      # config 1's size: standard layout, 1-row strips
    (300, 1088, 29),     # 17 words per row: standard, strips not dividing the rows
    (40, 64, 50),        # one word per row, fewer rows than 2k + strip
    (1024, 1024, 41),    # band, 2-row strips
    (100, 2048, 30),     # band, rows < 512
    (2000, 4096, 26),    # band, 3-4-row strips not dividing the rows
    (24, 1024, 25),      # band, the minimum rows for k = 12
    (777, 8192, 13),     # band, two column groups
])
def test_small_board_auto_strip_vs_oracle(G, H, W, turns):
    words = O.random_words(19 + H, 0, H, W // 64)
    ref, counts = O.bits_run(words, turns, with_counts=True)
    with G.Engine(H, W) as e:
        e.load_words(0, words)
        got = [int(c) for c in e.step_counted(turns, 12)]
        out = e.store_words(0, H)
    assert got == [int(c) for c in counts[11::12]]
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("H,W", [(8192, 8192), (4096, 4096), (512, 512)])
def test_small_board_auto_strip_vs_wide_strips(G, H, W):
    """Boards the oracle is slow on: the automatic (short) strips against explicit 96-row ones."""
    res = []
    for strip in (0, 96):
        with G.Engine(H, W, strip_rows=strip) as e:
            e.load_random(5)
            c = [int(x) for x in e.step_counted(12 * 9 + 7, 12)]
            res.append((c, e.hash()))
    assert res[0] == res[1]
