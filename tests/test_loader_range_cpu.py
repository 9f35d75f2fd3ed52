"""The pipeline loaders' interior-block range (gol_kernels.hip, band_pipe_kernel and
bytes_pipe_kernel `stage_in`), checked against the per-block test it replaced (no GPU).

A loader stages the blocks of its stream 0, 1, 2, ... (RPB rows each, walking down from
first_in or, for the upper walker of a paired range, up from s1e + K - 1).  A block whose rows
all lie inside [in_lo, in_hi] takes the carried row address; the others clamp per row.  Since
round 5 the kernels find the interior blocks once, as the range [ib_lo, ib_hi] from div_ceil_nn
/ div_floor, instead of comparing each block's rows; this restates both in Python and compares
them on every block of many stream shapes, including empty and one-block ranges."""
import itertools

import pytest


def div_ceil_nn(a, d):  # gol_kernels.hip div_ceil_nn: ceil(a / d) for a >= 0, else 0
    return (a + d - 1) // d if a > 0 else 0


def div_floor(a, d):  # gol_kernels.hip div_floor (C integer division, written for a < 0)
    return int(a / d) if a >= 0 else -((-a + d - 1) // d)


def interior_range(dir_, first_in, s1e, K, in_lo, in_hi, rpb):
    y_first = first_in if dir_ >= 0 else s1e + K - 1
    if dir_ >= 0:
        lo = div_ceil_nn(in_lo - y_first, rpb)
        hi = div_floor(in_hi - (rpb - 1) - y_first, rpb)
    else:
        lo = div_ceil_nn(y_first - in_hi, rpb)
        hi = div_floor(y_first - (rpb - 1) - in_lo, rpb)
    return lo, (hi - lo + 1 if hi >= lo else 0)


def per_block(dir_, first_in, s1e, K, in_lo, in_hi, rpb, b):  # round 4's test on the carried row
    y0 = first_in + rpb * b if dir_ >= 0 else s1e + K - 1 - rpb * b
    ylo, yhi = (y0, y0 + rpb - 1) if dir_ >= 0 else (y0 - (rpb - 1), y0)
    return ylo >= in_lo and yhi <= in_hi


@pytest.mark.parametrize("rpb,K", [(2, 12), (4, 32), (2, 8), (3, 12)])
def test_interior_range_matches_per_block_test(rpb, K):
    checked = 0
    for R, s0, n, dir_, contig in itertools.product([1, 7, 40, 1000], [0, 3, 17, 500], [1, 2, 5, 33, 600],
                                                   [1, 0, -1], [False, True]):
        s1 = min(R, s0 + n)
        if s0 >= s1:
            continue
        first_in, last_in = s0 - K, s1 + K - 1
        trip = rpb * 4
        s1e = s0 + ((s1 - s0 + 4 * K + trip - 1) // trip) * trip - 4 * K if dir_ else s1
        in_lo = first_in if contig else max(first_in, 0)
        in_hi = last_in if contig else min(last_in, R - 1)
        lo, cnt = interior_range(dir_, first_in, s1e, K, in_lo, in_hi, rpb)
        nblk = (s1e - s0 + 4 * K) // rpb + 8
        for b in range(nblk):
            want = per_block(dir_, first_in, s1e, K, in_lo, in_hi, rpb, b)
            got = 0 <= b - lo < cnt  # (uint32_t)(b - ib_lo) < ib_n
            assert got == want, (R, s0, s1, dir_, contig, b)
            checked += 1
    assert checked > 10000
