"""Wire types and RPC method names of the reference (stubs/stubs.go, util/cell.go).

gob matches fields by name, so these names are the ABI a Go drop-in keeps.
Boards are numpy uint8 arrays [y][x] here ([][]byte in Go).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import NamedTuple

import numpy as np

# stubs.go:5-11
GameOfLifeUpdate = "GameOfLifeOperations.Update"
Pause = "Operations.Pause"
Quit = "Operations.Quit"
SuperQuit = "Operations.SuperQuit"
BrokeOps = "Operations.Run"
Retrieve = "Operations.RetrieveCurrentData"
WorkerQuit = "GameOfLifeOperations.WorkerQuit"


class Cell(NamedTuple):  # util/cell.go:4-5
    X: int
    Y: int


@dataclass
class Parameters:  # stubs.go:13-18
    Turns: int = 0
    Threads: int = 0
    ImageWidth: int = 0
    ImageHeight: int = 0


@dataclass
class Request:  # stubs.go:20-29
    World: np.ndarray | None = None
    Turns: int = 0
    ImageHeight: int = 0
    ImageWidth: int = 0
    Threads: int = 0
    EndY: int = 0
    StartY: int = 0
    Worker: int = 0


@dataclass
class Response:  # stubs.go:31-38
    Alive: list = field(default_factory=list)
    AliveCount: int = 0
    TurnsCompleted: int = 0
    World: np.ndarray | None = None
    WorkSlice: np.ndarray | None = None
    Worker: int = 0
