"""The one-process-per-GPU rank engine (gol_engine_create_rank) with 2-4 processes on the one GPU
of the test box, over the IPC transport (RCCL refuses two ranks on one GPU): the product's own
halo plan, step plans, collectives (error words, counted-step series, load verdicts, PGM
barriers, the step-state agreement) and whole-board queries, with every rank a separate process
as under torch.distributed.run on an 8-GPU node.  broker.go:135-206's row split applied to GPU
ranks; the results are checked against the oracle, the golden PGM and the reference's alive CSV.

Each rank runs tests/_rank_worker.py; nothing here touches the GPU itself except through the
children.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "_rank_worker.py")
SPIN_LIB = os.path.join(ROOT, "gol-distributed-final_amd", "golhip", "libgolhip_spintest.so")


@pytest.fixture(scope="module")
def G():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import golhip
    golhip.lib()
    return golhip


def run_ranks(G, nranks, H, W, scenario, per_rank=None, timeout=150, ipc_timeout_ms=30000, transport="ipc", **kw):
    """Start nranks worker processes (one rank each) and return their JSON results by rank."""
    uid = G.engine.unique_id(transport).hex()
    kw["transport"] = transport
    env = dict(os.environ, GOL_IPC_TIMEOUT_MS=str(ipc_timeout_ms))
    procs = []
    for r in range(nranks):
        a = dict(kw, uid=uid, H=H, W=W, nranks=nranks, rank=r, scenario=scenario)
        if per_rank:
            a.update(per_rank(r))
        procs.append(subprocess.Popen([sys.executable, WORKER, json.dumps(a)], stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, env=env))
    res, errs = {}, []
    for p in procs:
        try:
            out, err = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            errs.append(f"rc {p.returncode}: {err[-3000:]}")
            continue
        d = json.loads(lines[-1])
        res[d["rank"]] = d
    assert not errs, "\n".join(errs)
    return res


def rows_sha(words):
    return hashlib.sha256(np.ascontiguousarray(words, dtype=np.uint64).tobytes()).hexdigest()


@pytest.mark.parametrize("nranks,H,W,k,turns,every", [
    (2, 1024, 2048, 0, 37, 5),     # band layout, k = 12 split pipeline; N = 2: both neighbours one peer
    (3, 1000, 2048, 0, 50, 12),    # uneven split (334 / 333 / 333)
    (4, 515, 4096, 0, 41, 1),      # uneven, a count after every turn
    (3, 301, 64 * 40, 8, 22, 11),  # standard layout (W % 1024 != 0), k = 8
    (4, 64, 1024, 0, 30, 10),      # 16-row shards: k capped at 12 by the halo, several launches
    (8, 1000, 2048, 0, 36, 12),    # N = 8 (config 5's rank count): the ring of 8, uneven rows (125 each)
])
def test_ipc_ranks_match_oracle(G, tmp_path, nranks, H, W, k, turns, every):
    ref, counts = O.bits_run(O.random_words(7, 0, H, W // 64), turns, with_counts=True)
    pgm = tmp_path / "ranks.pgm"
    res = run_ranks(G, nranks, H, W, "random", k=k, seed=7, turns=turns, every=every, pgm=str(pgm), flips=True)
    assert sorted(res) == list(range(nranks))
    after = O.bits_run(ref, 1)
    flips = O.flipped_cells(O.unpack(ref), O.unpack(after))
    for r, d in res.items():
        assert d["topology"] == {"shards": 1, "nranks": nranks, "rank": r, "transport": "ipc"}
        assert (d["y0"], d["y1"]) == G.partition_rows(H, nranks, r)
        assert d["counts"] == [int(counts[every * (i + 1) - 1]) for i in range(turns // every)]
        assert d["hash"] == O.hash_words(ref)
        assert d["alive"] == O.popcount_words(ref)
        assert d["rows_sha"] == rows_sha(ref[d["y0"]:d["y1"]])
        mine = [[x, y] for x, y in flips if d["y0"] <= y < d["y1"]]
        assert d["flips"] == mine
        assert d["hash_after_flip"] == O.hash_words(after)
    assert pgm.read_bytes() == O.pgm_bytes(O.unpack(ref))


@pytest.mark.parametrize("H,W,k,turns,every", [(1024, 2048, 0, 37, 5), (515, 4096, 0, 41, 1), (301, 64 * 40, 8, 22, 11)])
def test_rccl_ranks_match_oracle(G, tmp_path, H, W, k, turns, every):
    """RCCL between GPUs, one process per GPU as torch.distributed.run starts them (RCCL refuses two
    ranks on one GPU: needs >= 2 GPUs, skipped on a 1-GPU box): up to 8 ranks, the same checks as
    the IPC ranks' -- counts, hash, rows, the flipped cells and the P5 file against the oracle."""
    import torch
    n = min(torch.cuda.device_count(), 8)
    if n < 2:
        pytest.skip("RCCL ranks need >= 2 GPUs")
    ref, counts = O.bits_run(O.random_words(7, 0, H, W // 64), turns, with_counts=True)
    pgm = tmp_path / "ranks.pgm"
    res = run_ranks(G, n, H, W, "random", transport="rccl", per_rank=lambda r: {"device": r}, k=k, seed=7,
                    turns=turns, every=every, pgm=str(pgm), flips=True)
    after = O.bits_run(ref, 1)
    flips = O.flipped_cells(O.unpack(ref), O.unpack(after))
    for r, d in res.items():
        assert d["topology"] == {"shards": 1, "nranks": n, "rank": r, "transport": "rccl"}
        assert d["counts"] == [int(counts[every * (i + 1) - 1]) for i in range(turns // every)]
        assert d["hash"] == O.hash_words(ref)
        assert d["rows_sha"] == rows_sha(ref[d["y0"]:d["y1"]])
        assert d["flips"] == [[x, y] for x, y in flips if d["y0"] <= y < d["y1"]]
        assert d["hash_after_flip"] == O.hash_words(after)
    assert pgm.read_bytes() == O.pgm_bytes(O.unpack(ref))


@pytest.mark.parametrize("nranks", [2, 3])
def test_ipc_ranks_golden_512(G, golden_dir, tmp_path, nranks):
    """images/512x512.pgm, 100 turns (config 1), every rank streaming its rows from the file: the
    written PGM is check/images/512x512x100.pgm byte for byte, the count after every turn is
    check/alive/512.csv's, the alive list is the golden board's in row-major order."""
    out = tmp_path / "out.pgm"
    res = run_ranks(G, nranks, 512, 512, "pgm", path=os.path.join(golden_dir, "images", "512x512.pgm"),
                    turns=100, out=str(out))
    golden = open(os.path.join(golden_dir, "check", "images", "512x512x100.pgm"), "rb").read()
    assert out.read_bytes() == golden
    alive = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", "512x512.csv"))
    _, _, board = O.read_pgm(os.path.join(golden_dir, "check", "images", "512x512x100.pgm"))
    ys, xs = np.nonzero(board)
    for r, d in res.items():
        assert d["counts"] == [alive[t] for t in range(1, 101)]
        y0, y1 = d["y0"], d["y1"]
        sel = (ys >= y0) & (ys < y1)
        want = np.stack([xs[sel], ys[sel]], axis=1).astype(np.int32)
        assert d["ncells"] == len(want)
        assert d["cells_sha"] == hashlib.sha256(np.ascontiguousarray(want).tobytes()).hexdigest()


def test_ipc_load_words_on_one_rank(G):
    """load_words is not collective: one rank overwrites some of its rows, the other ranks do not
    call it.  The next stepping call's agreement makes every rank exchange its halo again, so the
    neighbours see the new rows (stale ghost rows / unmatched exchanges otherwise)."""
    H, W, turns = 600, 2048, 30
    base = O.random_words(3, 0, H, W // 64)
    y0, y1 = G.partition_rows(H, 3, 1)
    new = O.random_words(99, 0, 4, W // 64)
    wy0 = y0  # the first rows of rank 1: rank 0 reads them as its lower ghost rows
    board = base.copy()
    board[wy0:wy0 + 4] = new
    ref, counts = O.bits_run(board, turns, with_counts=True)
    res = run_ranks(G, 3, H, W, "loadwords", seed=3, turns=turns, every=10, writer=1, wy0=wy0,
                    words=[int(x) for x in new.ravel()])
    for d in res.values():
        assert d["hash"] == O.hash_words(ref)
        assert d["counts"] == [int(counts[9]), int(counts[19]), int(counts[29])]
        assert d["rows_sha"] == rows_sha(ref[d["y0"]:d["y1"]])


def test_ipc_fault_on_one_rank_fails_every_rank(G):
    """Rank 0 runs the spin-fault build (every pipeline flag wait times out at once), rank 1 the
    product library: the step fails with GOL_EHIP on BOTH ranks (the error words are all-reduced),
    and both work again afterwards."""
    if not os.path.exists(SPIN_LIB):
        pytest.skip("libgolhip_spintest.so not built")
    H, W = 400, 2048
    ref1 = O.bits_run(O.random_words(5, 0, H, W // 64), 1)
    res = run_ranks(G, 2, H, W, "fault", seed=5, turns=24, per_rank=lambda r: {"lib": SPIN_LIB} if r == 0 else {})
    for d in res.values():
        assert d["error"] is not None and d["error"][0] == G._lib.GOL_EHIP, d
        assert "timed out" in d["error"][1]
        assert d["hash1"] == O.hash_words(ref1)


def test_ipc_dead_rank_fails_the_others(G):
    """A rank that joins and then exits: the survivors' next collective fails (GOL_ECOMM / EHIP)
    within the IPC timeout instead of hanging."""
    res = run_ranks(G, 3, 300, 1024, "dead", victim=2, ipc_timeout_ms=4000, timeout=120)
    for r in (0, 1):
        err = res[r]["error"]
        assert err is not None and err[0] in (G._lib.GOL_ECOMM, G._lib.GOL_EHIP), res[r]


def test_ipc_bad_arguments(G):
    """IPC transport errors are codes, not crashes: no id, a non-IPC id, too many ranks."""
    with pytest.raises(G.GolError, match="bad rank arguments"):
        G.Engine.rank(64, 1024, 2, 0, None, device=0, transport="ipc")
    with pytest.raises(G.GolError, match="not an IPC id"):
        G.Engine.rank(64, 1024, 2, 0, bytes(128), device=0, transport="ipc")
    with pytest.raises(G.GolError, match="at most"):
        G.Engine.rank(64, 1024, 17, 0, G.engine.ipc_unique_id(), device=0, transport="ipc")


def test_ipc_one_rank(G):
    """One IPC rank: the halo is its own torus wrap, pulled from itself."""
    H, W = 150, 2048
    ref = O.bits_run(O.random_words(3, 0, H, W // 64), 40)
    with G.Engine.rank(H, W, 1, 0, G.engine.ipc_unique_id(), device=0, transport="ipc") as e:
        assert e.topology()["transport"] == "ipc"
        e.load_random(3)
        e.step(40)
        assert e.hash() == O.hash_words(ref)


def test_bench_share_gpu_shards_over_ipc(G):
    """`bench.py --gpus 2 --share-gpu` shards the weak board over 2 processes on this GPU (IPC
    transport, parallelism rows2): the alive count after the same turns equals the one-process
    run of the same 2x-row board."""
    def line(args):
        p = subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, capture_output=True, text=True, timeout=200)
        assert p.returncode == 0, p.stderr[-3000:]
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, p.stdout[-2000:]
        return json.loads(lines[0])
    common = ["--width", "65536", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--settle-s", "0"]
    two = line(["--gpus", "2", "--share-gpu", "--rows-per-gpu", "2048"] + common)
    one = line(["--rows-per-gpu", "4096"] + common)
    assert two["n_gpus"] == 2 and two["config"]["parallelism"] == "rows2" and two["config"]["transport"] == "ipc"
    assert two["config"]["H"] == one["config"]["H"] == 4096
    assert two["config"]["turns_done"] == one["config"]["turns_done"]
    assert two["config"]["alive_final"] == one["config"]["alive_final"]
    k = one["config"]["turns_per_step"]
    assert abs(two["value"] - 4096 * 65536 * k * 3 / (two["ms_per_step"] * 3e-3) / 1e9) < 0.02 * two["value"]
    # what each rank saw (bench.rank_stats): both ranks' engines report 2 ranks over IPC, the
    # warmup step's exchanges were timed on both ranks alike (the halo of the loaded board, then
    # the step's), and the per-rank step and exchange times are live event measurements
    rs = two["config"]["rank_stats"]
    assert rs["nranks_seen"] == [2, 2] and rs["transports"] == ["ipc"]
    n = rs["exchanges_per_rank"]
    assert n[0] == n[1] and 1 <= n[0] <= 2, n
    assert 0 < rs["launch_ms"]["min"] <= rs["launch_ms"]["max"]
    assert 0 < rs["exchange_ms"]["min"] <= rs["exchange_ms"]["max"]  # (the warmup's: incl. the first exchange)
    # its split (gol_engine_exchange_split): the IPC READY polls and the rest
    assert 0 <= rs["exchange_wait_ms"]["min"] <= rs["exchange_wait_ms"]["max"] <= rs["exchange_ms"]["max"]
    assert 0 < rs["exchange_transfer_ms"]["min"] <= rs["exchange_transfer_ms"]["max"]
    assert "rank_stats" not in one["config"]
    # every count of both runs against the reference series of the 4096 x 65536 board
    for d in (one, two):
        assert d["config"]["parity"]["status"] == "ok", d["config"]["parity"]
    assert two["config"]["parity"]["ranks"] == ["ok", "ok"]


def _bench(args, timeout=300):
    p = subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr[-3000:]


def test_bench_share_gpu_weak_board_parity(G):
    """The weak workload as the driver's N = 2 run sizes it (2 x 2^17 rows x 2^20, the default
    settle steps), 2 rank processes on this GPU over IPC: every alive count of the run equals one
    GPU's series of the same 2^18 x 2^20 torus (tests/golden/bench_counts.json)."""
    rc, d, err = _bench(["--gpus", "2", "--share-gpu", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"])
    assert rc == 0 and d, err
    assert d["config"]["H"] == 1 << 18 and d["config"]["parallelism"] == "rows2"
    par = d["config"]["parity"]
    assert par["status"] == "ok" and par["turns_checked"] == d["config"]["turns_done"], par


@pytest.mark.parametrize("n", [4, 8])
def test_bench_share_gpu_ring_parity(G, n):
    """The bench's rank ring at N = 4 and 8 (the driver's SCALE rank counts) on one GPU over IPC:
    4096 x 65536 split into N shares of 4096 / N rows -- the same torus as the N = 2 and the one-GPU
    runs -- every count of the run against its one-GPU series."""
    rc, d, err = _bench(["--gpus", str(n), "--share-gpu", "--rows-per-gpu", str(4096 // n), "--width", "65536",
                         "--steps", "6", "--warmup", "2", "--no-cpu-baseline", "--settle-s", "0"])
    assert rc == 0 and d, err
    par = d["config"]["parity"]
    assert d["config"]["parallelism"] == f"rows{n}" and par["status"] == "ok" and par["ranks"] == ["ok"] * n, par
    assert d["config"]["rank_stats"]["nranks_seen"] == [n] * n


def test_bench_mispaired_halo_fails_the_line(G):
    """A build whose ranks put each received halo block in the wrong ghost rows
    (libgolhip_mispair.so, GOL_TEST_MISPAIR) computes a plausible but wrong torus: bench.py's
    parity check names the first turn whose count differs and the run exits nonzero."""
    lib = os.path.join(ROOT, "gol-distributed-final_amd", "golhip", "libgolhip_mispair.so")
    if not os.path.exists(lib):
        pytest.skip("libgolhip_mispair.so not built (make -C gol-distributed-final_amd/csrc mispair)")
    rc, d, err = _bench(["--gpus", "2", "--share-gpu", "--rows-per-gpu", "2048", "--width", "65536", "--steps", "3",
                         "--warmup", "1", "--no-cpu-baseline", "--settle-s", "0", "--library", lib])
    assert rc == 1 and d, err
    par = d["config"]["parity"]
    assert par["status"] == "FAIL" and par["turn"] == 12 and par["got"] != par["want"], par
