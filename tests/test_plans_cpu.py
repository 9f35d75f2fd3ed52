"""The sharded step's schedule, as libgolhip.so exports it (host functions, no GPU).

gol_halo_plan is the one source of the halo exchange: the engine's exchange()
issues exactly these ops (ncclSend/ncclRecv in this order, or -- LOCAL/LOOPBACK --
device copies paired the way RCCL pairs them), and golhip.sharded's torch mirror
issues them as P2P ops.  Here the plans of every rank are executed on the CPU
with RCCL's matching rule (the n-th receive of rank b from rank a gets a's n-th
send to b) for 1..8 ranks and uneven splits, and every ghost row must end up
holding the right global row of the torus -- broker.go:135-206's partition with
the reference's row wrap (worker.go:48-59).  gol_step_plan must cover every row
once and flag exactly the launches that read ghost rows.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def G():
    import golhip
    golhip.lib()
    return golhip


def _run_plans(G, H, n, k):
    """Execute every rank's halo plan on numpy shards (value = global row index); returns the
    per-rank (top ghosts, bottom ghosts) after matching sends and receives RCCL's way."""
    parts = [G.partition_rows(H, n, r) for r in range(n)]
    plans = [G.halo_plan(H, n, r, k) for r in range(n)]
    shards = []
    for y0, y1 in parts:
        a = np.full(y1 - y0 + 2 * k, -1, dtype=np.int64)  # ghost rows [-k, 0) and [R, R + k)
        a[k:k + y1 - y0] = np.arange(y0, y1)
        shards.append(a)
    # queues of sends per (src, dst) in issue order
    sends = {}
    for r, plan in enumerate(plans):
        for kind, peer, row, rows in plan:
            if kind == "send":
                sends.setdefault((r, peer), []).append(shards[r][k + row:k + row + rows].copy())
    taken = {}
    for r, plan in enumerate(plans):
        for kind, peer, row, rows in plan:
            if kind == "recv":
                i = taken.get((peer, r), 0)
                taken[(peer, r)] = i + 1
                blk = sends[(peer, r)][i]
                assert len(blk) == rows
                shards[r][k + row:k + row + rows] = blk
    for key, q in sends.items():
        assert taken.get(key, 0) == len(q), f"unmatched sends {key}"
    return parts, shards


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("H,k", [(96, 12), (101, 8), (8 * 13 + 5, 12), (64, 1)])
def test_halo_plan_fills_every_ghost_row(G, n, H, k):
    if k > H // n:
        pytest.skip("k exceeds the smallest shard")
    parts, shards = _run_plans(G, H, n, k)
    for (y0, y1), a in zip(parts, shards):
        R = y1 - y0
        assert a[:k].tolist() == [(y0 - k + j) % H for j in range(k)]  # the k rows above, wrapped
        assert a[k + R:].tolist() == [(y1 + j) % H for j in range(k)]  # the k rows below, wrapped
        assert a[k:k + R].tolist() == list(range(y0, y1))              # own rows untouched


def test_halo_plan_two_ranks_same_peer_order(G):
    """nranks = 2: both neighbours are one peer; the issue order is what pairs the top rows
    with the peer's bottom ghost rows (gol_engine.cpp exchange(), ncclSend/ncclRecv)."""
    plan = G.halo_plan(64, 2, 0, 12)
    assert plan == [("send", 1, 0, 12), ("recv", 1, 32, 12), ("send", 1, 20, 12), ("recv", 1, -12, 12)]
    assert G.halo_plan(64, 1, 0, 4) == [("send", 0, 0, 4), ("recv", 0, 64, 4), ("send", 0, 60, 4), ("recv", 0, -4, 4)]


def test_halo_plan_errors(G):
    for args in [(10, 0, 0, 1), (10, 2, 2, 1), (10, 2, 0, 6), (10, 2, 0, 0), (3, 4, 0, 1)]:
        with pytest.raises(G.GolError):
            G.halo_plan(*args)


@pytest.mark.parametrize("mode", ["overlap", "edge_first", "serial"])
@pytest.mark.parametrize("R,k,kx", [(1000, 12, 12), (1000, 1, 12), (36, 12, 12), (35, 12, 12), (13, 8, 12),
                                    (5, 1, 1), (3, 1, 1), (2, 1, 1)])
def test_step_plan_covers_rows_once(G, R, k, kx, mode):
    if kx > R:
        pytest.skip("kx > R")
    plan = G.step_plan(R, k, kx, mode)
    split = mode != "serial" and R >= 3 * kx
    cover = np.zeros(R, dtype=int)
    for stream, needs_halo, row0, rows in plan:
        cover[row0:row0 + rows] += 1
        reads_ghosts = row0 - k < 0 or row0 + rows + k > R
        assert needs_halo == reads_ghosts, (stream, row0, rows)
        assert (stream == "edge") == (split and mode == "overlap" and needs_halo)
    assert (cover == 1).all()
    if split:
        # the rows the next exchange sends are written by the launches that read the halo, all
        # of them before the interior in launch order
        halo = np.zeros(R, dtype=bool)
        for stream, needs_halo, row0, rows in plan:
            if needs_halo:
                halo[row0:row0 + rows] = True
        assert halo[:kx].all() and halo[R - kx:].all() and not halo[kx:R - kx].any()
        assert [h for _, h, _, _ in plan] == [True, True, False]
    else:
        assert plan == [("main", True, 0, R)]
