"""Wire types and RPC method names of the reference (stubs/stubs.go, util/cell.go).

gob matches fields by name, so these names are the ABI a Go drop-in keeps.
Boards are numpy uint8 arrays [y][x] here ([][]byte in Go).
"""
from __future__ import annotations

from collections.abc import Sequence
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


class CellList(Sequence):
    """The alive list of a Response ([]util.Cell, broker.go:47-58) as the (n, 2) int32 (x, y)
    pairs the device wrote, row-major; a Cell is made when an element is read.  Building a
    Python list of n Cells costs ~1.3 us per cell (0.6 s for a 4096^2 board's 481k cells), far
    more than the Run itself, so a Response holds the pairs and converts on access."""
    __slots__ = ("_xy",)

    def __init__(self, xy=()):
        self._xy = np.asarray(xy, dtype=np.int32).reshape(-1, 2)

    def __len__(self) -> int:
        return len(self._xy)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return CellList(self._xy[i])
        x, y = self._xy[i].tolist()
        return Cell(x, y)

    def __iter__(self):
        return map(Cell._make, self._xy.tolist())

    def __eq__(self, other):
        if isinstance(other, CellList):
            return np.array_equal(self._xy, other._xy)
        if isinstance(other, Sequence):
            return len(self) == len(other) and all(a == b for a, b in zip(self, other))
        return NotImplemented

    def __repr__(self) -> str:
        return f"CellList({list(self)!r})" if len(self) <= 8 else f"CellList(<{len(self)} cells>)"

    def array(self) -> np.ndarray:
        """The (n, 2) int32 (x, y) pairs."""
        return self._xy


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
