"""A Game-of-Life board resident in HBM (ctypes wrapper of gol_engine_*).

Replaces the broker's per-turn board handling (broker.go:62-234): the board is
loaded once into HBM and stepped in k-turn kernel launches; queries (alive
count, alive list, the board bytes, a PGM snapshot) are served from the device.
The board may be row-sharded over several GPUs (broker.go:135-206's partition
applied to GPUs) with a k-row halo exchange per launch: `shards=` in one process
(RCCL between distinct GPUs, device copies between shards sharing a GPU), or
`Engine.rank(...)` with one process per GPU (RCCL; or HIP IPC between the processes of one node,
which may share a GPU).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import (GOL_EINVAL, GOL_IPC_ID_BYTES, GOL_RCCL_ID_BYTES, GOL_SHARDS_SAME_DEVICE, GOL_TIMING_EXCHANGE,
                   GOL_WRITE_FN, LAYOUTS, STEP_MODES, TRANSPORT_NAMES, TRANSPORTS, GolError, check, gol_config, lib)


def rccl_unique_id(library=None) -> bytes:
    """A fresh RCCL unique id (gol_rccl_unique_id) for Engine.rank; share it with every rank."""
    L = library or lib()
    buf = (ctypes.c_uint8 * GOL_RCCL_ID_BYTES)()
    rc = L.gol_rccl_unique_id(buf, GOL_RCCL_ID_BYTES)
    if rc:
        raise GolError(rc, L.gol_last_error().decode(errors="replace"))
    return bytes(buf)


def ipc_unique_id(library=None) -> bytes:
    """A fresh id for Engine.rank(..., transport="ipc") (gol_ipc_unique_id: host only, no GPU);
    share it with every rank."""
    L = library or lib()
    buf = (ctypes.c_uint8 * GOL_IPC_ID_BYTES)()
    rc = L.gol_ipc_unique_id(buf, GOL_IPC_ID_BYTES)
    if rc:
        raise GolError(rc, L.gol_last_error().decode(errors="replace"))
    return bytes(buf)


def unique_id(transport: str = "rccl", library=None) -> bytes:
    """The id Engine.rank needs for `transport` ("rccl" or "ipc")."""
    return ipc_unique_id(library) if transport == "ipc" else rccl_unique_id(library)


class Engine:
    def __init__(self, height: int, width: int, *, turns_per_launch: int = 0, cells_per_lane: int = 0,
                 strip_rows: int = 0, device: int = -1, layout: str = "auto", shards: int = 1,
                 transport: str = "auto", same_device: bool = False, step: str = "auto", library=None, _rank=None):
        self.H, self.W = int(height), int(width)
        self._L = library or lib()
        cfg = gol_config(device=device, turns_per_launch=turns_per_launch, strip_rows=strip_rows,
                         cells_per_lane=cells_per_lane, layout=LAYOUTS[layout], shards=shards,
                         transport=TRANSPORTS[transport],
                         flags=(GOL_SHARDS_SAME_DEVICE if same_device else 0) | STEP_MODES[step])
        h = ctypes.c_void_p()
        if _rank is None:
            self._check(self._L.gol_engine_create(self.H, self.W, ctypes.byref(cfg), ctypes.byref(h)))
        else:
            nranks, rank, uid = _rank
            idbuf = None
            if uid is not None:
                # the C side reads exactly GOL_RCCL_ID_BYTES (= GOL_IPC_ID_BYTES) bytes of the id: a
                # shorter buffer would be read past its end
                if len(uid) != GOL_RCCL_ID_BYTES or len(uid) != GOL_IPC_ID_BYTES:
                    raise GolError(GOL_EINVAL, f"rank id must be {GOL_RCCL_ID_BYTES} bytes, got {len(uid)}")
                idbuf = (ctypes.c_uint8 * GOL_RCCL_ID_BYTES).from_buffer_copy(uid)
            self._check(self._L.gol_engine_create_rank(self.H, self.W, nranks, rank, idbuf, ctypes.byref(cfg),
                                                       ctypes.byref(h)))
        self._h = h

    @classmethod
    def rank(cls, height: int, width: int, nranks: int, rank: int, uid: bytes | None, **kw) -> "Engine":
        """This process's shard `rank` of an `nranks`-rank board (collective: every rank constructs
        it with the same uid).  transport="rccl" (default with nranks > 1: one process per GPU, uid
        from rccl_unique_id) or "ipc" (processes of one node that may share a GPU, uid from
        ipc_unique_id)."""
        return cls(height, width, _rank=(nranks, rank, uid), **kw)

    def _check(self, rc: int) -> None:
        if rc:
            raise GolError(rc, self._L.gol_last_error().decode(errors="replace"))

    # -- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            self._L.gol_engine_destroy(self._h)
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
        self._check(self._L.gol_engine_load_bytes(self._h, world.ctypes.data, self.W))

    def load_random(self, seed: int) -> None:
        self._check(self._L.gol_engine_load_random(self._h, seed))

    def load_pgm(self, path: str) -> None:
        """readPgmImage (gol/io.go:90-126): every shard streams its own rows of the file."""
        self._check(self._L.gol_engine_load_pgm(self._h, path.encode()))

    def store_bytes(self) -> np.ndarray:
        out = np.empty((self.H, self.W), dtype=np.uint8)
        self._check(self._L.gol_engine_store_bytes(self._h, out.ctypes.data, self.W))
        return out

    def store_rows(self, y0: int, y1: int) -> np.ndarray:
        out = np.empty((max(y1 - y0, 0), self.W), dtype=np.uint8)
        self._check(self._L.gol_engine_store_rows(self._h, y0, y1, out.ctypes.data, self.W))
        return out

    def write_pgm(self, path: str) -> None:
        self._check(self._L.gol_engine_write_pgm(self._h, path.encode()))

    def write_pgm_to(self, sink) -> None:
        """The P5 byte stream (gol/io.go:52-81) into sink(offset, memoryview) instead of a file:
        the header, then chunks of rows in row order (this process's rows, at their file
        offsets).  The memoryview is only valid during the call."""
        err = []

        def cb(_user, off, data, n):
            try:
                sink(off, (ctypes.c_uint8 * n).from_address(data))
                return 0
            except BaseException as x:  # noqa: BLE001 -- reported after the call
                err.append(x)
                return 1
        fn = GOL_WRITE_FN(cb)
        rc = self._L.gol_engine_write_pgm_to(self._h, fn, None)
        if err:
            raise err[0]
        self._check(rc)

    def load_words(self, y0: int, words: np.ndarray) -> None:
        """Rows [y0, y0 + len(words)) from bit-packed uint64 rows (64 cells per word, LSB = lowest x)."""
        words = np.ascontiguousarray(words, dtype=np.uint64)
        if words.ndim != 2 or words.shape[1] != self.W // 64:
            raise ValueError(f"expected (rows, {self.W // 64}) uint64 words")
        self._check(self._L.gol_engine_load_words(self._h, y0, y0 + words.shape[0], words.ctypes.data, words.shape[1]))

    def store_words(self, y0: int, y1: int) -> np.ndarray:
        out = np.empty((max(y1 - y0, 0), self.W // 64), dtype=np.uint64)
        self._check(self._L.gol_engine_store_words(self._h, y0, y1, out.ctypes.data, self.W // 64))
        return out

    # -- stepping and queries
    def step(self, turns: int) -> None:
        self._check(self._L.gol_engine_step(self._h, turns))

    def step_counted(self, turns: int, every: int) -> np.ndarray:
        """Advance `turns` turns; the alive count after every `every` turns (fused on the GPU)."""
        n = turns // every if every > 0 else 0
        out = np.zeros(max(n, 1), dtype=np.uint64)
        self._check(self._L.gol_engine_step_counted(self._h, turns, every, out.ctypes.data, n))
        return out[:n]

    @property
    def turn(self) -> int:
        t = ctypes.c_int64()
        self._check(self._L.gol_engine_turn(self._h, ctypes.byref(t)))
        return t.value

    def alive_count(self) -> int:
        c = ctypes.c_uint64()
        self._check(self._L.gol_engine_alive_count(self._h, ctypes.byref(c)))
        return c.value

    def alive_cells(self, cap: int | None = None) -> np.ndarray:
        """(n, 2) int32 array of (x, y) in row-major order (broker.go:47-58)."""
        if cap is None:
            cap = self.alive_count()
        xy = np.zeros((max(cap, 1), 2), dtype=np.int32)
        n = ctypes.c_int64()
        self._check(self._L.gol_engine_alive_cells(self._h, xy.ctypes.data, cap, ctypes.byref(n)))
        return xy[:min(n.value, cap)]

    def step_flips(self, cap: int | None = None) -> np.ndarray:
        """Advance one turn; (n, 2) int32 (x, y) of the cells that changed, row-major: the
        CellFlipped events of that turn (gol/event.go:50-60)."""
        if cap is None:
            cap = self.H * self.W
        xy = np.zeros((max(cap, 1), 2), dtype=np.int32)
        n = ctypes.c_int64()
        self._check(self._L.gol_engine_step_flips(self._h, xy.ctypes.data, cap, ctypes.byref(n)))
        return xy[:min(n.value, cap)]

    def hash(self) -> int:
        h = ctypes.c_uint64()
        self._check(self._L.gol_engine_hash(self._h, ctypes.byref(h)))
        return h.value

    def info(self) -> dict:
        k, cpl, strip, bm = (ctypes.c_int32() for _ in range(4))
        self._check(self._L.gol_engine_info(self._h, ctypes.byref(k), ctypes.byref(cpl), ctypes.byref(strip),
                                    ctypes.byref(bm)))
        return {"turns_per_launch": k.value, "cells_per_lane": cpl.value, "strip_rows": strip.value,
                "bit_mode": bool(bm.value), "layout": {0: "bytes", 1: "standard", 2: "band"}[bm.value]}

    def topology(self) -> dict:
        s, n, r, t = (ctypes.c_int32() for _ in range(4))
        self._check(self._L.gol_engine_topology(self._h, ctypes.byref(s), ctypes.byref(n), ctypes.byref(r),
                                                ctypes.byref(t)))
        return {"shards": s.value, "nranks": n.value, "rank": r.value, "transport": TRANSPORT_NAMES[t.value]}

    def shard(self, i: int) -> dict:
        d, a, b = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self._L.gol_engine_shard(self._h, i, ctypes.byref(d), ctypes.byref(a), ctypes.byref(b)))
        return {"device": d.value, "y0": a.value, "y1": b.value}

    def set_timing(self, enable: bool, exchanges: bool = False) -> None:
        """HIP-event timing of the stepping calls; exchanges=True also times every halo exchange
        of them (GOL_TIMING_EXCHANGE: one event pair each, on the stream it runs on)."""
        level = (GOL_TIMING_EXCHANGE if exchanges else 1) if enable else 0
        self._check(self._L.gol_engine_set_timing(self._h, level))

    def exchange_timing(self) -> dict:
        """Halo exchanges timed since set_timing(True, exchanges=True): their mean duration, and
        its split (gol_engine_exchange_split) into the wait for the ring neighbours to reach the
        exchange and the transfer of the halo rows."""
        n, ms, w, x = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        self._check(self._L.gol_engine_exchange_timing(self._h, ctypes.byref(n), ctypes.byref(ms)))
        self._check(self._L.gol_engine_exchange_split(self._h, ctypes.byref(n), ctypes.byref(w), ctypes.byref(x)))
        return {"exchanges": n.value, "mean_ms": ms.value, "wait_ms": w.value, "transfer_ms": x.value}

    def timing(self) -> dict:
        """HIP-event timing of every shard-step since set_timing(True) (edge launches included)."""
        n, ms, cells = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        self._check(self._L.gol_engine_timing(self._h, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(cells)))
        return {"launches": n.value, "mean_ms": ms.value, "mean_cell_updates": cells.value}

    def device_bits(self):
        p = ctypes.c_void_p()
        pitch = ctypes.c_int64()
        self._check(self._L.gol_engine_device_bits(self._h, ctypes.byref(p), ctypes.byref(pitch)))
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
