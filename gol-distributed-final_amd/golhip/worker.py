"""The worker's RPC service `GameOfLifeOperations` (worker.go:73-86) over the C ABI."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, gol_request, gol_response, lib
from .stubs import Request, Response


class GameOfLifeOperations:
    def Update(self, req: Request) -> Response:
        """worker.go:77-80: res.WorkSlice = calculateNextState(StartY, EndY, World)."""
        world = np.ascontiguousarray(req.World, dtype=np.uint8)
        H, W = world.shape
        r = gol_request(World=world.ctypes.data, world_stride=W, Turns=req.Turns, ImageHeight=H,
                        ImageWidth=W, Threads=req.Threads, EndY=req.EndY, StartY=req.StartY,
                        Worker=req.Worker)
        out = np.empty((max(req.EndY - req.StartY, 0), W), dtype=np.uint8)
        res = gol_response(WorkSlice=out.ctypes.data, work_stride=W)
        check(lib().gol_worker_update(ctypes.byref(r), ctypes.byref(res)))
        return Response(WorkSlice=out, Worker=res.Worker)

    def WorkerQuit(self, req: Request | None = None) -> Response:
        """worker.go:82-86: the Go drop-in closes its listener; nothing to free here."""
        return Response()
