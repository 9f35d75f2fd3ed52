"""The bit-sliced B3/S23 circuit of the gfx950 kernels, checked on the CPU over every 3x3
neighbourhood (worker.go:26-37 / 44-70 semantics on 0/255 cells).

gol_kernels.hip computes a generation from the three rows' horizontal 3-sums (h0 = xor3,
h1 = maj of a cell and its two horizontal neighbours; the centre row's sum includes the cell)
with 7 three-input gates (v_bitop3_b32): t0, k0 (low bits), u, v (high bits), then the tail
found by tools/rule_search.c: G1 = TT_G1(t0, k0, v), G2 = TT_G2(u, v, G1),
alive' = TT_OUT(t0, cell, G2).  The truth tables are read from the kernel source, so this test
fails if the source's gates stop computing the rule.
"""
import itertools
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gol-distributed-final_amd", "csrc", "gol_kernels.hip")


def _tables():
    text = open(SRC).read()
    tt = {m.group(1): int(m.group(2), 16) for m in re.finditer(r"constexpr unsigned (TT_\w+) = 0x([0-9A-Fa-f]+);", text)}
    for name in ("TT_XOR3", "TT_MAJ", "TT_G1", "TT_G2", "TT_OUT"):
        assert name in tt, name
    return tt


def _gate(tt, a, b, c):
    # v_bitop3_b32 convention: operand 0 -> 0xF0, operand 1 -> 0xCC, operand 2 -> 0xAA
    return (tt >> ((a << 2) | (b << 1) | c)) & 1


def test_rule_circuit_is_b3s23_on_every_neighbourhood():
    T = _tables()
    assert _gate(T["TT_XOR3"], 1, 1, 0) == 0 and _gate(T["TT_MAJ"], 1, 1, 0) == 1
    for nb in itertools.product((0, 1), repeat=9):
        rows = [nb[0:3], nb[3:6], nb[6:9]]
        h = [sum(r) for r in rows]                      # horizontal 3-sums, centre row incl. the cell
        lo, hi = [x & 1 for x in h], [x >> 1 for x in h]
        t0 = _gate(T["TT_XOR3"], *lo)
        k0 = _gate(T["TT_MAJ"], *lo)
        u = _gate(T["TT_XOR3"], *hi)
        v = _gate(T["TT_MAJ"], *hi)
        g1 = _gate(T["TT_G1"], t0, k0, v)
        g2 = _gate(T["TT_G2"], u, v, g1)
        got = _gate(T["TT_OUT"], t0, nb[4], g2)
        n = sum(nb) - nb[4]
        want = 1 if (n == 3 or (nb[4] == 1 and n == 2)) else 0   # B3/S23
        assert got == want, nb


def test_rule_circuit_needs_the_centre_sum_to_include_the_cell():
    """The 3-gate tail relies on the centre row's sum including the cell (tools/rule_search.c
    finds no 3-gate tail without that don't-care): feeding it a centre sum without the cell is
    wrong somewhere -- a guard against reusing the tail on neighbour-only sums."""
    T = _tables()
    wrong = 0
    for nb in itertools.product((0, 1), repeat=9):
        rows = [list(nb[0:3]), list(nb[3:6]), list(nb[6:9])]
        h = [sum(rows[0]), rows[1][0] + rows[1][2], sum(rows[2])]
        lo, hi = [x & 1 for x in h], [x >> 1 for x in h]
        t0, k0 = _gate(T["TT_XOR3"], *lo), _gate(T["TT_MAJ"], *lo)
        u, v = _gate(T["TT_XOR3"], *hi), _gate(T["TT_MAJ"], *hi)
        got = _gate(T["TT_OUT"], t0, nb[4], _gate(T["TT_G2"], u, v, _gate(T["TT_G1"], t0, k0, v)))
        n = sum(nb) - nb[4]
        wrong += got != (1 if (n == 3 or (nb[4] == 1 and n == 2)) else 0)
    assert wrong > 0


def _pair_tables():
    text = open(SRC).read()
    tt = {m.group(1): int(m.group(2), 16) for m in re.finditer(r"constexpr unsigned (TT_\w+) = 0x([0-9A-Fa-f]+);", text)}
    for name in ("TT_PG1", "TT_PG2", "TT_PG3", "TT_POUT"):
        assert name in tt, name
    return tt


def _life(rows):
    n = sum(sum(r) for r in rows) - rows[1][1]
    return 1 if (n == 3 or (rows[1][1] == 1 and n == 2)) else 0


def _pair_step(T, rows):
    """gol_kernels.hip pstage on one column: rows = 4 x 3 cells (x_2m-2, x_2m-1, x_2m, x_2m+1),
    the outputs of rows 2m-1 and 2m."""
    h = [sum(r) for r in rows]
    a, b, c, d = [(x & 1, x >> 1) for x in h]
    k = b[0] & c[0]
    p0 = b[0] ^ c[0]
    p1 = _gate(T["TT_XOR3"], b[1], c[1], k)
    p2 = _gate(T["TT_MAJ"], b[1], c[1], k)

    def tail(x0, x1, cell):
        g1 = _gate(T["TT_PG1"], p0, x0, cell)
        g2 = _gate(T["TT_PG2"], p1, p2, x1)
        g3 = _gate(T["TT_PG3"], p2, cell, g1)
        return _gate(T["TT_POUT"], g3, g1, g2)
    return (p0 + 2 * p1 + 4 * p2, tail(a[0], a[1], rows[1][1]), tail(d[0], d[1], rows[2][1]))


def test_pair_circuit_is_b3s23_on_every_neighbourhood():
    """The band pipeline's pair step (tools/rule_search_pair.c): the shared
    binary pair sum of the two middle rows and the two 4-gate tails give B3/S23 for both output
    rows on all 4096 4 x 3 neighbourhoods."""
    T = _pair_tables()
    for nb in itertools.product((0, 1), repeat=12):
        rows = [nb[0:3], nb[3:6], nb[6:9], nb[9:12]]
        P, o0, o1 = _pair_step(T, rows)
        assert P == sum(rows[1]) + sum(rows[2])
        assert o0 == _life(rows[0:3]), nb
        assert o1 == _life(rows[1:4]), nb


def test_pair_tail_needs_the_cell_row_in_the_pair():
    """The 4-gate tail uses the don't-cares of a cell whose row is one of the pair (P >= 1 for a
    live cell, <= 5 for a dead one): over all (P, x, cell) it is wrong somewhere -- a guard
    against feeding it a pair that excludes the cell's row."""
    T = _pair_tables()
    wrong = 0
    for P in range(7):
        for x in range(4):
            for cell in (0, 1):
                p0, p1, p2 = P & 1, (P >> 1) & 1, P >> 2
                g1 = _gate(T["TT_PG1"], p0, x & 1, cell)
                g2 = _gate(T["TT_PG2"], p1, p2, x >> 1)
                out = _gate(T["TT_POUT"], _gate(T["TT_PG3"], p2, cell, g1), g1, g2)
                t = P + x
                wrong += out != (1 if (t == 3 or (cell and t == 4)) else 0)
    assert wrong > 0
