"""CPU checks of bench.py's orchestration (no GPU): the self-launch of N ranks over gloo,
the one-line JSON contract, and the roofline bookkeeping (a PMC profile measured on another
gol_kernels.hip is never used)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_self_launch_two_ranks_dry_run():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dry-run", "--steps", "4"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    # rank 0's stdout is the one JSON line and nothing else (gloo's "[Gloo] Rank 0 is connected"
    # message goes to stderr): a driver may read the first line
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["ranks"] == 2
    # max over ranks: rank 1 reported 2 ms, rank 0 1 ms
    assert abs(d["ms_per_step"] - 2.0 / 4) < 1e-6
    for key in ("metric", "value", "unit", "steps", "warmup", "higher_is_better", "scaling", "vs_baseline", "dtype",
                "data", "config", "roofline", "cpu_baseline"):
        assert key in d
    # N > 1: what each rank saw (bench.rank_stats), so one multi-GPU run separates compute
    # imbalance (launch_ms spread) from exchange cost (exchange_ms); the dry run's fake per-rank
    # numbers: rank r steps (r + 1) / steps ms, exchanges 0.01 (r + 1) ms
    rs = d["config"]["rank_stats"]
    assert rs["launch_ms"] == {"max": 0.5, "min": 0.25}
    assert rs["exchange_ms"] == {"max": 0.02, "min": 0.01}
    # its split: the wait for the ring neighbours and the transfer (gol_engine_exchange_split)
    assert rs["exchange_wait_ms"] == {"max": 0.008, "min": 0.004}
    assert rs["exchange_transfer_ms"] == {"max": 0.012, "min": 0.006}
    assert rs["wall_ms"] == {"max": 2.0, "min": 1.0}
    assert rs["nranks_seen"] == [2, 2] and rs["exchanges_per_rank"] == [20, 20]  # (the warmup's: weak's default 20)
    assert rs["transports"] == ["dry-run"] and "basis" in rs


def test_self_launch_ends_when_a_rank_dies():
    """A rank that dies leaves its peers blocked in a collective with it: the launcher must not
    wait for them forever -- it terminates the survivors and returns the failure."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--dry-run", "--fail-rank", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert time.monotonic() - t0 < 60
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dry-run"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE=3" in p.stderr


def test_roofline_uses_only_current_profiles(tmp_path, monkeypatch):
    current = bench.kernel_source_hash()
    entry = {"kernel_src": current, "bytes_per_launch": 3.5e10, "valu_insts_per_launch": 9.0e9,
             "profile": "profiles/x"}
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_traffic.json").write_text(json.dumps({"a": entry, "b": dict(entry, kernel_src="0" * 16)}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    pmc, note = bench.load_pmc("a")
    assert pmc is not None and note == "profiles/x"
    r = bench.roofline("bits", 12.0, 131072 * 1048576 * 12, pmc, note)
    assert r["bound"] == "valu"
    assert abs(r["frac"] - 9.0e9 / 12e-3 / 1e9 / bench.VALU_PEAK_GINST) < 1e-4
    assert abs(r["hbm"]["frac"] - 3.5e10 / 12e-3 / 1e9 / 8000) < 1e-4
    assert abs(r["effective_GBs"] - 0.25 * 131072 * 1048576 * 12 / 12e-3 / 1e9) < 0.1
    stale, why = bench.load_pmc("b")
    assert stale is None and why.startswith("stale")
    r = bench.roofline("bits", 12.0, 1e12, None, "missing")
    assert r["bound"] == "hbm" and r["frac"] is None and r["traffic"] is None


class _OneRank:
    world, rank = 1, 0

    def gather(self, obj):
        return [obj]


def test_parity_check_against_reference_series(tmp_path, monkeypatch):
    """bench.parity: every count of the run against the reference series of its board; a
    mismatch names the first turn that differs, a run longer than the series is 'partial', a
    board without a series 'unpinned'."""
    fx = tmp_path / "counts.json"
    fx.write_text(json.dumps({"boards": {"8x64": {"every": 4, "counts": [10, 11, 12, 13]}}}))
    monkeypatch.setattr(bench, "COUNTS_FIXTURE", str(fx))
    r = _OneRank()
    assert bench.parity(r, "8x64", 4, [10, 11, 12])["status"] == "ok"
    bad = bench.parity(r, "8x64", 4, [10, 11, 99, 13])
    assert bad["status"] == "FAIL" and bad["turn"] == 12 and bad["got"] == 99 and bad["want"] == 12
    assert bench.parity(r, "8x64", 4, [10, 11, 12, 13, 14])["status"] == "partial"
    assert bench.parity(r, "8x64", 8, [11])["status"] == "unpinned"
    assert bench.parity(r, "16x64", 4, [1])["status"] == "unpinned"
    # and against the CPU oracle's series (tests/golden/oracle_counts.json) over the turns it holds
    orc = tmp_path / "oracle.json"
    orc.write_text(json.dumps({"boards": {"8x64": {"every": 4, "counts": [10, 11]}}}))
    monkeypatch.setattr(bench, "ORACLE_COUNTS", str(orc))
    ok = bench.parity(r, "8x64", 4, [10, 11, 12])
    assert ok["status"] == "ok" and ok["oracle"]["status"] == "ok" and ok["oracle"]["turns_checked"] == 8
    orc.write_text(json.dumps({"boards": {"8x64": {"every": 4, "counts": [10, 12]}}}))
    bad = bench.parity(r, "8x64", 4, [10, 11, 12])
    assert bad["status"] == "FAIL" and bad["oracle"]["status"] == "FAIL" and bad["turn"] == 8


def _fixture():
    with open(bench.COUNTS_FIXTURE) as f:
        return json.load(f)["boards"]


def test_reference_series_cover_the_bench_runs():
    """tests/golden/bench_counts.json holds a series for every board bench.py times -- the weak
    board at 1/2/4/8 ranks (the driver's SCALE runs), 262144^2 at any rank count, 65536^2 and the
    byte board -- long enough for the default runs and the driver's --steps 20 --warmup 5."""
    boards = _fixture()

    def need(workload, world, steps, warmup):
        a = bench.parse(["--workload", workload, "--gpus", str(world)] +
                        (["--steps", str(steps), "--warmup", str(warmup)] if steps else []))
        if workload == "byte16k":
            H = W = 16384
            k, rate, per_rank = 32, bench.SETTLE_RATE_BYTES, H * W
        else:
            H, W = {"weak": (a.rows_per_gpu * world, a.width), "strong262k": (262144, 262144),
                    "bit64k": (65536, 65536)}[workload]
            k, rate = 12, bench.SETTLE_RATE_BITS
            per_rank = (H // world if workload in ("weak", "strong262k") else H) * W
        settle = bench.settle_steps(a, lambda n: None, float(per_rank) * k, rate)
        return f"{H}x{W}", k, settle + a.warmup + a.steps

    for workload, worlds in (("weak", (1, 2, 4, 8)), ("strong262k", (1, 2, 4, 8)), ("bit64k", (1,)), ("byte16k", (1,))):
        for world in worlds:
            for steps, warmup in ((None, None), (20, 5)):
                key, k, points = need(workload, world, steps, warmup)
                assert key in boards, key
                assert boards[key]["every"] == k and len(boards[key]["counts"]) >= points, (key, points)


def test_reference_series_start_as_the_oracle():
    """The first points of two series against the oracle's word-parallel run of the same
    load_random(1) board (the rest: tiled-oracle GPU tests pin the kernels that made them)."""
    from oracle import oracle as O
    boards = _fixture()
    for key, H, W, turns in (("16384x16384", 16384, 16384, 32), ("4096x65536", 4096, 65536, 24)):
        s = boards[key]
        _, rc = O.bits_run(O.random_words(1, 0, H, W // 64), turns, with_counts=True)
        e = s["every"]
        assert s["counts"][:turns // e] == [int(rc[e * (i + 1) - 1]) for i in range(turns // e)]
