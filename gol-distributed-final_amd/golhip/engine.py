"""A Game-of-Life board resident on one MI355X (ctypes wrapper of gol_engine_*).

Replaces the broker's per-turn board handling (broker.go:62-234): the board is
loaded once into HBM and stepped in k-turn kernel launches; queries (alive
count, alive list, the board bytes, a PGM snapshot) are served from the device.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import LAYOUTS, check, gol_config, lib


class Engine:
    def __init__(self, height: int, width: int, *, turns_per_launch: int = 0, cells_per_lane: int = 0,
                 strip_rows: int = 0, device: int = -1, layout: str = "auto"):
        self.H, self.W = int(height), int(width)
        cfg = gol_config(device=device, turns_per_launch=turns_per_launch, strip_rows=strip_rows,
                         cells_per_lane=cells_per_lane, layout=LAYOUTS[layout])
        h = ctypes.c_void_p()
        check(lib().gol_engine_create(self.H, self.W, ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h

    # -- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            lib().gol_engine_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- board in / out
    def load_bytes(self, world: np.ndarray) -> None:
        world = np.ascontiguousarray(world, dtype=np.uint8)
        if world.shape != (self.H, self.W):
            raise ValueError(f"board shape {world.shape} != {(self.H, self.W)}")
        check(lib().gol_engine_load_bytes(self._h, world.ctypes.data, self.W))

    def load_random(self, seed: int) -> None:
        check(lib().gol_engine_load_random(self._h, seed))

    def store_bytes(self) -> np.ndarray:
        out = np.empty((self.H, self.W), dtype=np.uint8)
        check(lib().gol_engine_store_bytes(self._h, out.ctypes.data, self.W))
        return out

    def write_pgm(self, path: str) -> None:
        check(lib().gol_engine_write_pgm(self._h, path.encode()))

    # -- stepping and queries
    def step(self, turns: int) -> None:
        check(lib().gol_engine_step(self._h, turns))

    @property
    def turn(self) -> int:
        t = ctypes.c_int64()
        check(lib().gol_engine_turn(self._h, ctypes.byref(t)))
        return t.value

    def alive_count(self) -> int:
        c = ctypes.c_uint64()
        check(lib().gol_engine_alive_count(self._h, ctypes.byref(c)))
        return c.value

    def alive_cells(self, cap: int | None = None) -> np.ndarray:
        """(n, 2) int32 array of (x, y) in row-major order (broker.go:47-58)."""
        if cap is None:
            cap = self.alive_count()
        xy = np.zeros((max(cap, 1), 2), dtype=np.int32)
        n = ctypes.c_int64()
        check(lib().gol_engine_alive_cells(self._h, xy.ctypes.data, cap, ctypes.byref(n)))
        return xy[:min(n.value, cap)]

    def step_flips(self, cap: int | None = None) -> np.ndarray:
        """Advance one turn; (n, 2) int32 (x, y) of the cells that changed, row-major: the
        CellFlipped events of that turn (gol/event.go:50-60)."""
        if cap is None:
            cap = self.H * self.W
        xy = np.zeros((max(cap, 1), 2), dtype=np.int32)
        n = ctypes.c_int64()
        check(lib().gol_engine_step_flips(self._h, xy.ctypes.data, cap, ctypes.byref(n)))
        return xy[:min(n.value, cap)]

    def hash(self) -> int:
        h = ctypes.c_uint64()
        check(lib().gol_engine_hash(self._h, ctypes.byref(h)))
        return h.value

    def info(self) -> dict:
        k, cpl, strip, bm = (ctypes.c_int32() for _ in range(4))
        check(lib().gol_engine_info(self._h, ctypes.byref(k), ctypes.byref(cpl), ctypes.byref(strip),
                                    ctypes.byref(bm)))
        return {"turns_per_launch": k.value, "cells_per_lane": cpl.value, "strip_rows": strip.value,
                "bit_mode": bool(bm.value), "layout": {0: None, 1: "standard", 2: "band"}[bm.value]}

    def device_bits(self):
        p = ctypes.c_void_p()
        pitch = ctypes.c_int64()
        check(lib().gol_engine_device_bits(self._h, ctypes.byref(p), ctypes.byref(pitch)))
        return p.value, pitch.value


def next_state_slab(world: np.ndarray, start_y: int, end_y: int) -> np.ndarray:
    """worker.go:15-42 calculateNextState(startY, endY, world) on the GPU."""
    world = np.ascontiguousarray(world, dtype=np.uint8)
    H, W = world.shape
    out = np.empty((max(end_y - start_y, 0), W), dtype=np.uint8)
    check(lib().gol_next_state_slab(world.ctypes.data, H, W, W, start_y, end_y, out.ctypes.data, W))
    return out


def partition_rows(height: int, parts: int, i: int) -> tuple[int, int]:
    """broker.go:135-139 / 172-206 row split -> (StartY, EndY)."""
    a, b = ctypes.c_int64(), ctypes.c_int64()
    check(lib().gol_partition_rows(height, parts, i, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value
