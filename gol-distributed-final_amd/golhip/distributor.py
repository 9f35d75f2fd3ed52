"""Controller mirror: gol.Run + distributor (gol/gol.go:11-41, gol/distributor.go:24-185).

The reference's controller stays Go and unchanged in a real deployment (it talks to the
broker over net/rpc).  This module restates its behaviour over the same broker API
(`Run`, `RetrieveCurrentData`, `Pause`, `Quit`, `SuperQuit`) so the reference's
end-to-end tests (gol_test.go, pgm_test.go, count_test.go) can be replayed against the
GPU broker in-process, without a Go toolchain:

* the main thread reads images/<W>x<H>.pgm, calls ``ops.Run`` (blocking), then sends
  FinalTurnComplete, writes out/<W>x<H>x<Turns>.pgm, sends ImageOutputComplete and
  StateChange(Quitting) and closes the event stream (distributor.go:134-185);
* a ticker thread calls ``RetrieveCurrentData`` every ``tick`` seconds (2 s in the
  reference) and sends AliveCellsCount unless paused, and serves key presses
  (distributor.go:24-131): 's' saves the board, 'q' saves it, sends StateChange(Quitting)
  and calls Quit, 'k' the same with SuperQuit, 'p' toggles Pause and sends
  StateChange(Paused) / StateChange(Executing) with ``TurnsCompleted - 1`` on resume
  (distributor.go:118, kept).

Events go to a ``queue.Queue``; ``None`` marks the closed channel (close(c.events)).
CellFlipped / TurnComplete exist (event.go:50-63) but the reference's distributor never
sends them; ``Engine.step_flips`` produces them for a live view.
"""
from __future__ import annotations

import enum
import os
import queue
import threading
import time
from dataclasses import dataclass, field

from .pgm import read_pgm, write_pgm_bytes
from .stubs import Cell, Parameters, Request


class State(enum.IntEnum):  # event.go:32-40
    Paused = 0
    Executing = 1
    Quitting = 2

    def __str__(self) -> str:  # event.go:72-83
        return self.name


@dataclass(frozen=True)
class AliveCellsCount:  # event.go:19-24
    CompletedTurns: int
    CellsCount: int

    def GetCompletedTurns(self) -> int:
        return self.CompletedTurns


@dataclass(frozen=True)
class ImageOutputComplete:  # event.go:26-30
    CompletedTurns: int
    Filename: str

    def GetCompletedTurns(self) -> int:
        return self.CompletedTurns


@dataclass(frozen=True)
class StateChange:  # event.go:42-46
    CompletedTurns: int
    NewState: State

    def GetCompletedTurns(self) -> int:
        return self.CompletedTurns


@dataclass(frozen=True)
class CellFlipped:  # event.go:50-54
    CompletedTurns: int
    Cell: Cell

    def GetCompletedTurns(self) -> int:
        return self.CompletedTurns


@dataclass(frozen=True)
class TurnComplete:  # event.go:58-61
    CompletedTurns: int

    def GetCompletedTurns(self) -> int:
        return self.CompletedTurns


@dataclass(frozen=True)
class FinalTurnComplete:  # event.go:65-68
    CompletedTurns: int
    Alive: list = field(default_factory=list)

    def GetCompletedTurns(self) -> int:
        return self.CompletedTurns


def events_of(q: "queue.Queue", timeout: float | None = None):
    """Iterate a run's events until the stream is closed (`for event := range events`)."""
    while True:
        e = q.get(timeout=timeout)
        if e is None:
            return
        yield e


def _write_image(out_dir: str, name: str, world) -> None:
    """io.go:42-87 writePgmImage: out/<name>.pgm (the directory is created if missing)."""
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, name + ".pgm"), "wb") as f:
        f.write(write_pgm_bytes(world))


def _ticker(p: Parameters, events, key_presses, ops, done: threading.Event, request: Request, out_dir: str,
            tick: float) -> None:
    """distributor.go:24-131 tickerFunc."""
    request2 = Request(Turns=p.Turns, ImageHeight=p.ImageHeight, ImageWidth=p.ImageWidth, Threads=p.Threads)
    out_name = f"{p.ImageWidth}x{p.ImageHeight}x{p.Turns}"
    pause = False
    next_tick = time.monotonic() + tick
    while not done.is_set():
        wait = min(max(next_tick - time.monotonic(), 0.0), 0.05)
        key = None
        if key_presses is not None:
            try:
                key = key_presses.get(timeout=wait)
            except queue.Empty:
                pass
        else:
            time.sleep(wait)
        if done.is_set():
            break
        if key is None:
            if time.monotonic() < next_tick:
                continue
            next_tick += tick
            r = ops.RetrieveCurrentData(request2, alive=False, world=False)
            if not pause:
                events.put(AliveCellsCount(r.TurnsCompleted, r.AliveCount))
        elif key in ("q", "k"):
            r = ops.RetrieveCurrentData(request, alive=False)
            _write_image(out_dir, out_name, r.World)
            events.put(StateChange(r.TurnsCompleted, State.Quitting))
            done.set()
            if key == "q":
                ops.Quit(request)
            else:
                ops.SuperQuit(request)
        elif key == "s":
            r = ops.RetrieveCurrentData(request, alive=False)
            _write_image(out_dir, out_name, r.World)
        elif key == "p":
            r = ops.RetrieveCurrentData(request, alive=False, world=False)
            if not pause:
                events.put(StateChange(r.TurnsCompleted, State.Paused))
                ops.Pause(request)
                pause = True
            else:
                events.put(StateChange(r.TurnsCompleted - 1, State.Executing))  # distributor.go:118
                ops.Pause(request)
                pause = False


def run(p: Parameters, events: "queue.Queue", key_presses: "queue.Queue | None", *, ops,
        images_dir: str = "images", out_dir: str = "out", tick: float = 2.0) -> None:
    """gol.Run(p, events, keyPresses) (gol/gol.go:11-41 + distributor.go:133-185).  Blocks
    until the run is over and the stream closed; run it in a thread to consume events live."""
    world = read_pgm(os.path.join(images_dir, f"{p.ImageWidth}x{p.ImageHeight}.pgm"), p.ImageWidth,
                     p.ImageHeight)
    request = Request(World=world, Turns=p.Turns, ImageHeight=p.ImageHeight, ImageWidth=p.ImageWidth,
                      Threads=p.Threads)
    done = threading.Event()
    ticker = threading.Thread(target=_ticker, args=(p, events, key_presses, ops, done, request, out_dir, tick),
                              daemon=True)
    ticker.start()
    try:
        response = ops.Run(request)
        turn = response.TurnsCompleted
        events.put(FinalTurnComplete(turn, list(response.Alive)))
        out_name = f"{p.ImageWidth}x{p.ImageHeight}x{p.Turns}"
        _write_image(out_dir, out_name, response.World)
        events.put(ImageOutputComplete(response.TurnsCompleted, out_name))
        events.put(StateChange(turn, State.Quitting))
    finally:
        done.set()
        ticker.join()
        events.put(None)  # close(c.events)
