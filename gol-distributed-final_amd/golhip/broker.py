"""The broker's RPC service `Operations` (broker.go:62-277) over the C ABI.

``Operations`` keeps the reference's method names and argument meaning; the
work is done by the C++ service object in libgolhip.so (gol_host.cpp), which
keeps the board resident on the GPU instead of scattering it to workers every
turn.  Errors come back as ``GolError`` instead of a panic.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import LAYOUTS, TRANSPORTS, check, gol_config, gol_request, gol_response, lib
from .stubs import CellList, Request, Response


def _request(req: Request, keep: list) -> gol_request:
    r = gol_request()
    if req.World is not None:
        world = np.ascontiguousarray(req.World, dtype=np.uint8)
        if world.ndim != 2 or world.shape != (req.ImageHeight, req.ImageWidth):
            # the reference indexes World[y][x] for y < ImageHeight, x < ImageWidth and would
            # panic on a smaller board (broker.go:67-70, 96-105)
            raise ValueError(f"World has shape {world.shape}, expected (ImageHeight, ImageWidth) = "
                             f"{(req.ImageHeight, req.ImageWidth)}")
        keep.append(world)
        r.World = world.ctypes.data
        r.world_stride = world.shape[1]
    r.Turns, r.ImageHeight, r.ImageWidth = req.Turns, req.ImageHeight, req.ImageWidth
    r.Threads, r.EndY, r.StartY, r.Worker = req.Threads, req.EndY, req.StartY, req.Worker
    return r


def _cells(xy: np.ndarray, n: int) -> CellList:
    return CellList(xy[:n].copy())  # the copy lets the H*W-pair buffer go


class Operations:
    """broker.go:60 `type Operations struct{}` with its five RPC methods."""

    def __init__(self, *, device: int = -1, turns_per_launch: int = 0, cells_per_lane: int = 0, shards: int = 1,
                 transport: str = "auto", same_device: bool = False, layout: str = "auto"):
        """shards > 1: the board of a Run is row-sharded over that many GPUs (the reference's
        Threads split, broker.go:135-206, applied to GPUs), with the same results.  layout="bytes":
        the board stays one byte per cell on one GPU (GOL_LAYOUT_BYTES, the byte pipeline)."""
        cfg = gol_config(device=device, turns_per_launch=turns_per_launch, cells_per_lane=cells_per_lane,
                         shards=shards, transport=TRANSPORTS[transport], flags=1 if same_device else 0,
                         layout=LAYOUTS[layout])
        h = ctypes.c_void_p()
        check(lib().gol_broker_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().gol_broker_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _call(self, fn, req: Request, alive: bool, world: bool) -> Response:
        keep: list = []
        r = _request(req, keep)
        H, W = req.ImageHeight, req.ImageWidth
        res = gol_response()
        out_world = np.zeros((H, W), dtype=np.uint8) if world else None
        cap = H * W if alive else 0
        xy = np.zeros((max(cap, 1), 2), dtype=np.int32)
        if out_world is not None:
            res.World = out_world.ctypes.data
            res.world_stride = W
        if alive:
            res.Alive = xy.ctypes.data
            res.alive_cap = cap
        check(fn(self._h, ctypes.byref(r), ctypes.byref(res)))
        return Response(Alive=_cells(xy, res.alive_len) if alive else [], AliveCount=res.AliveCount,
                        TurnsCompleted=res.TurnsCompleted, World=out_world)

    def Run(self, req: Request) -> Response:  # broker.go:62-234
        return self._call(lib().gol_broker_run, req, alive=True, world=True)

    def RetrieveCurrentData(self, req: Request, *, alive: bool = True, world: bool = True) -> Response:
        """broker.go:256-277.  ``alive=False`` / ``world=False`` skip the list / board copy
        (the count is always returned)."""
        return self._call(lib().gol_broker_retrieve, req, alive=alive, world=world)

    def Pause(self, req: Request | None = None) -> Response:  # broker.go:251-254
        check(lib().gol_broker_pause(self._h))
        return Response()

    def Quit(self, req: Request | None = None) -> Response:  # broker.go:236-239
        check(lib().gol_broker_quit(self._h))
        return Response()

    def SuperQuit(self, req: Request | None = None) -> Response:  # broker.go:241-249
        check(lib().gol_broker_superquit(self._h))
        return Response()

    @property
    def paused(self) -> bool:
        p = ctypes.c_int32()
        check(lib().gol_broker_paused(self._h, ctypes.byref(p)))
        return bool(p.value)
