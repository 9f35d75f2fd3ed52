"""The controller mirror (golhip.distributor: gol/gol.go + gol/distributor.go) replaying the
reference's end-to-end tests.

* CPU: the controller logic against an oracle-backed stand-in for the broker (test
  infrastructure only, like the gloo tests' kernel stand-in): event order, file output,
  ticker, key presses.
* GPU: the reference's own test matrix through the controller and the GPU broker
  (golhip.Operations): TestGol gol_test.go:15-47, TestPgm pgm_test.go:10-42, TestAlive
  count_test.go:17-69.
"""
import os
import queue
import threading
import time

import numpy as np
import pytest

from oracle import oracle as O


def _golden_cells(golden_dir, size, turns):
    """gol_test.go:88-129 readAliveCells: every nonzero byte of the golden image."""
    _, _, g = O.read_pgm(os.path.join(golden_dir, "check", "images", f"{size}x{size}x{turns}.pgm"))
    ys, xs = np.nonzero(g)
    return sorted(zip(xs.tolist(), ys.tolist()))


def _run_async(D, p, ops, images, out, keys=None, tick=2.0):
    ev = queue.Queue()
    th = threading.Thread(target=D.run, args=(p, ev, keys), daemon=True,
                          kwargs=dict(ops=ops, images_dir=images, out_dir=out, tick=tick))
    th.start()
    return ev, th


class OracleOps:
    """Broker stand-in (tests only): the broker.go:62-277 contract over the numpy oracle, one
    turn at a time; Quit ends Run, Pause toggles, Retrieve returns a consistent snapshot."""

    def __init__(self, turn_delay=0.0):
        self.lock = threading.Lock()
        self.turn, self.world = 0, None
        self.quit = self.paused = False
        self.superquit = False
        self.delay = turn_delay

    def Run(self, req):
        from golhip.stubs import Cell, Response
        world = np.array(req.World, dtype=np.uint8)
        with self.lock:
            self.turn, self.world, self.quit = 0, world.copy(), False
        t = 0
        while t < req.Turns:
            with self.lock:
                if self.quit:
                    break
                if self.paused:
                    pass
            if self.paused:
                time.sleep(0.001)
                continue
            world = O.np_next_state(world)
            t += 1
            with self.lock:
                self.turn, self.world = t, world.copy()
            if self.delay:
                time.sleep(self.delay)
        ys, xs = np.nonzero(world)
        return Response(Alive=[Cell(int(x), int(y)) for x, y in zip(xs, ys)], TurnsCompleted=t, World=world)

    def RetrieveCurrentData(self, req, alive=True, world=True):
        from golhip.stubs import Response
        with self.lock:
            w = self.world.copy() if self.world is not None else np.zeros((req.ImageHeight, req.ImageWidth), np.uint8)
            return Response(AliveCount=int(np.count_nonzero(w)), TurnsCompleted=self.turn, World=w if world else None)

    def Pause(self, req=None):
        with self.lock:
            self.paused = not self.paused

    def Quit(self, req=None):
        with self.lock:
            self.quit = True

    def SuperQuit(self, req=None):
        self.superquit = True
        self.Quit()


# ------------------------------------------------------------------ CPU: controller logic
def test_events_and_output_order(golden_dir, tmp_path):
    from golhip import distributor as D
    from golhip.stubs import Parameters
    p = Parameters(Turns=100, Threads=4, ImageWidth=16, ImageHeight=16)
    ev, th = _run_async(D, p, OracleOps(), os.path.join(golden_dir, "images"), str(tmp_path))
    events = list(D.events_of(ev, timeout=60))
    th.join(10)
    final = [e for e in events if isinstance(e, D.FinalTurnComplete)]
    assert len(final) == 1 and final[0].CompletedTurns == 100
    assert sorted((c.X, c.Y) for c in final[0].Alive) == _golden_cells(golden_dir, 16, 100)
    tail = events[-3:]
    assert isinstance(tail[0], D.FinalTurnComplete)
    assert tail[1] == D.ImageOutputComplete(100, "16x16x100")
    assert tail[2] == D.StateChange(100, D.State.Quitting)
    with open(tmp_path / "16x16x100.pgm", "rb") as f:
        got = f.read()
    with open(os.path.join(golden_dir, "check", "images", "16x16x100.pgm"), "rb") as f:
        assert got == f.read()


def test_ticker_and_keys(golden_dir, tmp_path):
    """AliveCellsCount every tick; 'p' pauses (no counts while paused), 'p' resumes with the
    TurnsCompleted - 1 quirk (distributor.go:118); 's' saves; 'q' saves, quits the run."""
    from golhip import distributor as D
    from golhip.stubs import Parameters
    p = Parameters(Turns=10**9, Threads=2, ImageWidth=64, ImageHeight=64)
    keys = queue.Queue()
    ops = OracleOps(turn_delay=0.0005)
    ev, th = _run_async(D, p, ops, os.path.join(golden_dir, "images"), str(tmp_path), keys, tick=0.05)
    expected = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", "64x64.csv"))
    counts = []
    for e in D.events_of(ev, timeout=30):
        assert isinstance(e, D.AliveCellsCount)
        if e.CompletedTurns:
            assert e.CellsCount == expected[e.CompletedTurns]
        counts.append(e)
        if len(counts) == 3:
            break
    keys.put("p")
    e = ev.get(timeout=30)
    while isinstance(e, D.AliveCellsCount):  # ticks that raced the key press
        e = ev.get(timeout=30)
    assert isinstance(e, D.StateChange) and e.NewState == D.State.Paused
    time.sleep(0.3)
    paused_at = ops.turn  # Retrieve runs before Pause (distributor.go:111-113): the event may lag
    assert e.CompletedTurns <= paused_at
    assert ev.empty()  # no AliveCellsCount while paused
    keys.put("s")
    time.sleep(0.2)
    saved = O.read_pgm(str(tmp_path / "64x64x1000000000.pgm"))[2]
    keys.put("p")
    e = ev.get(timeout=30)
    assert e.NewState == D.State.Executing and e.CompletedTurns == paused_at - 1
    assert np.array_equal(saved, O.run(O.read_pgm(os.path.join(golden_dir, "images", "64x64.pgm"))[2], paused_at))
    keys.put("q")
    rest = list(D.events_of(ev, timeout=30))
    th.join(10)
    quits = [e for e in rest if isinstance(e, D.StateChange)]
    assert [q.NewState for q in quits] == [D.State.Quitting, D.State.Quitting]
    final = [e for e in rest if isinstance(e, D.FinalTurnComplete)][0]
    assert paused_at < final.CompletedTurns < 10**9
    assert rest[-2] == D.ImageOutputComplete(final.CompletedTurns, "64x64x1000000000")


def test_superquit_key(golden_dir, tmp_path):
    from golhip import distributor as D
    from golhip.stubs import Parameters
    keys = queue.Queue()
    ops = OracleOps(turn_delay=0.001)
    ev, th = _run_async(D, Parameters(Turns=10**9, Threads=1, ImageWidth=16, ImageHeight=16), ops,
                        os.path.join(golden_dir, "images"), str(tmp_path), keys, tick=10.0)
    while ops.turn < 5:
        time.sleep(0.01)
    keys.put("k")
    events = list(D.events_of(ev, timeout=30))
    th.join(10)
    assert ops.superquit
    assert events[0].NewState == D.State.Quitting
    assert isinstance(events[1], D.FinalTurnComplete)


# ------------------------------------------------------------------ GPU: the reference's tests
@pytest.fixture(scope="module")
def gpu_ops():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import golhip as G
    ops = G.Operations(device=0)
    yield ops
    ops.close()


@pytest.mark.gpu
@pytest.mark.parametrize("size", [16, 64, 512])
@pytest.mark.parametrize("turns", [0, 1, 100])
def test_gol_and_pgm_through_controller(gpu_ops, golden_dir, tmp_path, size, turns):
    """TestGol (FinalTurnComplete.Alive == golden alive cells) and TestPgm (out/<W>x<H>x<T>.pgm
    == golden, byte for byte) for 1..16 threads."""
    from golhip import distributor as D
    from golhip.stubs import Parameters
    want = _golden_cells(golden_dir, size, turns)
    with open(os.path.join(golden_dir, "check", "images", f"{size}x{size}x{turns}.pgm"), "rb") as f:
        want_pgm = f.read()
    for threads in range(1, 17):
        p = Parameters(Turns=turns, Threads=threads, ImageWidth=size, ImageHeight=size)
        out = tmp_path / str(threads)
        ev, th = _run_async(D, p, gpu_ops, os.path.join(golden_dir, "images"), str(out))
        events = list(D.events_of(ev, timeout=60))
        th.join(10)
        final = [e for e in events if isinstance(e, D.FinalTurnComplete)]
        assert len(final) == 1 and final[0].CompletedTurns == turns
        assert sorted((c.X, c.Y) for c in final[0].Alive) == want, f"threads={threads}"
        with open(out / f"{size}x{size}x{turns}.pgm", "rb") as f:
            assert f.read() == want_pgm, f"threads={threads}"


@pytest.mark.gpu
def test_alive_through_controller(gpu_ops, golden_dir, tmp_path):
    """TestAlive (count_test.go:17-69): 512x512, 10^8 turns, 8 threads; the first 5
    AliveCellsCount events match check/alive (or 5565/5567 past turn 10000); then 'q'."""
    from golhip import distributor as D
    from golhip.stubs import Parameters
    expected = O.read_alive_csv(os.path.join(golden_dir, "check", "alive", "512x512.csv"))
    p = Parameters(Turns=100000000, Threads=8, ImageWidth=512, ImageHeight=512)
    keys = queue.Queue()
    ev, th = _run_async(D, p, gpu_ops, os.path.join(golden_dir, "images"), str(tmp_path), keys, tick=0.25)
    n = 0
    for e in D.events_of(ev, timeout=5):  # "no AliveCellsCount events received in 5 seconds"
        if isinstance(e, D.AliveCellsCount):
            t = e.CompletedTurns
            want = expected[t] if 0 < t <= 10000 else (0 if t == 0 else (5565 if t % 2 == 0 else 5567))
            assert e.CellsCount == want, f"turn {t}"
            n += 1
        if n >= 5:
            keys.put("q")
            break
    rest = list(D.events_of(ev, timeout=60))
    th.join(30)
    assert not th.is_alive()
    final = [e for e in rest if isinstance(e, D.FinalTurnComplete)][0]
    t = final.CompletedTurns
    assert 0 < t < 100000000
    assert len(final.Alive) == (expected[t] if t <= 10000 else (5565 if t % 2 == 0 else 5567))
