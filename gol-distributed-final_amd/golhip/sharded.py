"""torch.distributed mirror of the row-sharded step -- one process per rank.

The product's sharded board is libgolhip.so's engine (gol_engine_create_rank: RCCL halo
exchange inside the library, golhip.Engine.rank).  This module runs the SAME schedule with
torch.distributed point-to-point ops, so that it can be driven on the CPU with the gloo
backend (tests/test_sharded_gloo.py) or with several ranks sharing one GPU: the halo plan
(gol_halo_plan) and the step plan (gol_step_plan) come from the library, not from here.

The reference splits the board into `Threads` row slabs per turn and ships the WHOLE board
to every worker each turn (broker.go:135-206, 143-157).  Here the partition
(gol_partition_rows, broker.go:172-206) is applied once: rank r keeps rows [y0_r, y1_r) and,
per k-turn step, computes the edge rows (which read the kmax halo rows) and the interior,
then exchanges the new edge rows with its ring neighbours.

Counts and hashes are per-shard reductions summed with one all_reduce.  PyTorch provides
device memory, the stream and torch.distributed only; all board arithmetic runs in
libgolhip.so's gfx950 kernels (or, in the CPU tests, an oracle stand-in).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from ._lib import GOL_COUNT_SLOTS, check, halo_plan, lib, step_plan
from .engine import partition_rows

VALID_K = (16, 12, 8, 4, 2, 1)


class HipKernels:
    """Launch the C-ABI device kernels on torch CUDA tensors and torch's current stream."""

    def __init__(self, cells_per_lane: int = 0, strip_rows: int = 0, band_cells_per_lane: int = 0):
        self.cells_per_lane = cells_per_lane
        self.band_cells_per_lane = band_cells_per_lane  # 0 = library default
        self.strip_rows = strip_rows
        lib()  # fail loudly now if the library is missing

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    def bits_step(self, top, mid, bot, dst, row0: int, rows: int, k: int, slots=None) -> None:
        R, pitch = mid.shape
        check(lib().gol_dev_bits_step(top.data_ptr(), mid.data_ptr(), bot.data_ptr(), dst.data_ptr(), R,
                                      self.Wd, pitch, row0, rows, k, self.cells_per_lane, self.strip_rows,
                                      slots.data_ptr() if slots is not None else None, self._stream()))

    def band_step(self, top, mid, bot, dst, row0: int, rows: int, k: int, slots=None) -> None:
        R, pitch = mid.shape
        check(lib().gol_dev_band_step(top.data_ptr(), mid.data_ptr(), bot.data_ptr(), dst.data_ptr(), R,
                                      self.Wd, pitch, row0, rows, k, self.band_cells_per_lane, self.strip_rows,
                                      slots.data_ptr() if slots is not None else None, self._stream()))

    def band_max_k(self) -> int:
        return lib().gol_band_max_k(self.band_cells_per_lane)

    def band_convert(self, to_band: bool, src, dst) -> None:
        check(lib().gol_dev_band_convert(1 if to_band else 0, src.data_ptr(), dst.data_ptr(), src.shape[0], self.Wd,
                                         src.shape[1], dst.shape[1], self._stream()))

    def random_fill(self, dst, grow0: int, W: int, seed: int) -> None:
        rows, pitch = dst.shape
        check(lib().gol_dev_random_fill(dst.data_ptr(), rows, grow0, W, pitch, seed, self._stream()))

    def popcount(self, src, slots) -> None:
        rows, pitch = src.shape
        check(lib().gol_dev_popcount(src.data_ptr(), rows, self.Wd, pitch, slots.data_ptr(), self._stream()))

    def hash(self, src, grow0: int, slots) -> None:
        rows, pitch = src.shape
        check(lib().gol_dev_hash(src.data_ptr(), rows, grow0, self.Wd, pitch, slots.data_ptr(), self._stream()))

    def unpack(self, src, W: int) -> torch.Tensor:
        rows, pitch = src.shape
        out = torch.empty((rows, W), dtype=torch.uint8, device=src.device)
        check(lib().gol_dev_unpack(src.data_ptr(), rows, W, pitch, out.data_ptr(), W, self._stream()))
        return out

    def pack(self, board, dst, nonbinary=None) -> None:
        """0/255 bytes -> bits; nonbinary (int32 device tensor) gets 1 if any byte is neither."""
        rows, W = board.shape
        check(lib().gol_dev_pack(board.data_ptr(), rows, W, W, dst.data_ptr(), dst.shape[1],
                                 nonbinary.data_ptr() if nonbinary is not None else None, self._stream()))


class ShardedBoard:
    """A W-wide, H-tall bit-packed torus, rows sharded over the ranks of `group`."""

    def __init__(self, height: int, width: int, *, turns_per_launch: int = 0, cells_per_lane: int = 0,
                 strip_rows: int = 0, device=None, kernels=None, group=None, layout: str = "auto"):
        if width % 64:
            raise ValueError("the sharded bit board needs W % 64 == 0")
        if layout not in ("auto", "standard", "band"):
            raise ValueError(f"unknown layout {layout!r}")
        if layout == "band" and width % 1024:
            raise ValueError("the band layout needs W % 1024 == 0")
        self.H, self.W = int(height), int(width)
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank, self.nranks = dist.get_rank(group), dist.get_world_size(group)
        else:
            self.rank, self.nranks = 0, 1
        self.y0, self.y1 = partition_rows(self.H, self.nranks, self.rank)
        self.R = self.y1 - self.y0
        min_rows = self.H // self.nranks  # smallest shard (broker.go:172-206 split)
        if min_rows < 1:
            raise ValueError(f"{self.nranks} ranks cannot shard {self.H} rows")
        self.Wd = self.W // 32
        self.pitch = (self.Wd + 3) // 4 * 4
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if kernels is None else torch.device("cpu")
        self.device = torch.device(device)
        self.kern = kernels if kernels is not None else HipKernels(cells_per_lane, strip_rows)
        # Band layout: stepped shift-free; converted back before any read.
        self.use_band = layout != "standard" and self.W % 1024 == 0 and hasattr(self.kern, "band_step")
        if layout == "band" and not self.use_band:
            raise ValueError("these kernels have no band-layout step")
        kcap = self.kern.band_max_k() if self.use_band and hasattr(self.kern, "band_max_k") else (8 if self.use_band else 16)
        # k = 12 exists only as the band layout's split pipeline (4 words per lane)
        self.valid_k = tuple(k for k in VALID_K if k != 12 or kcap == 12)
        if turns_per_launch <= 0:  # library defaults: 12 on the band layout (split pipeline), else 8
            turns_per_launch = 12 if (self.use_band and kcap == 12) else 8
        self.kmax = max(k for k in self.valid_k if k <= max(1, min(turns_per_launch, min_rows, kcap)))
        self.band = False  # buf[cur] holds the band layout
        self.kern.Wd = self.Wd
        z = dict(dtype=torch.int32, device=self.device)
        # Each buffer keeps kmax halo rows right above and below the shard's R rows, so the
        # halo (received from the neighbours, or the torus wrap on one rank) is contiguous
        # with the board: the band kernel then addresses row y as board + y*pitch.
        self._store = [torch.zeros((self.R + 2 * self.kmax, self.pitch), **z) for _ in range(2)]
        self.buf = [t[self.kmax:self.kmax + self.R] for t in self._store]
        self.cur = 0
        self.halo_ok = False  # the ghost rows of buf[cur] hold the current halo (kmax rows)
        self.slots = torch.zeros(GOL_COUNT_SLOTS * 8, dtype=torch.int64, device=self.device)
        self.turn = 0
        # per-launch hooks (tests): called as hook("edge"|"main", k, rows, before)
        self.launch_hook = None

    # ------------------------------------------------------------ board in/out
    @property
    def board(self) -> torch.Tensor:
        return self.buf[self.cur]

    def load_random(self, seed: int) -> None:
        """Synthetic torus: identical global board for every rank count."""
        self.kern.random_fill(self.board, self.y0, self.W, seed)
        self.band = False
        self.halo_ok = False
        self.turn = 0

    def _convert(self, to_band: bool) -> None:
        if self.band == to_band:
            return
        self.kern.band_convert(to_band, self.board, self.buf[1 - self.cur])
        self.cur = 1 - self.cur
        self.halo_ok = False
        self.band = to_band

    def standard(self) -> torch.Tensor:
        """This rank's rows in the standard bit layout (converts back from the band layout)."""
        self._convert(False)
        return self.board

    def load_bytes(self, board_rows) -> None:
        """Load this rank's rows [y0, y1) from a (R, W) uint8 tensor of 0/255 bytes."""
        if tuple(board_rows.shape) != (self.R, self.W):
            raise ValueError("expected this rank's (R, W) rows")
        self.kern.pack(board_rows.to(self.device).contiguous(), self.board)
        self.band = False
        self.halo_ok = False
        self.turn = 0

    def load_pgm(self, path: str, chunk_rows: int = 4096) -> None:
        """Stream this rank's rows [y0, y1) of a P5 image (gol/io.go:90-126 header rules) into
        the shard: memory-mapped row chunks -> device -> packed, so no rank holds more than one
        chunk of bytes.  The reference's images are 0/255; other bytes need the exact first
        turn of the single-GPU engine (worker.go:26-37) and are rejected here."""
        from .pgm import pgm_rows
        rows = pgm_rows(path, self.y0, self.y1, self.W, self.H)
        flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        for a in range(0, self.R, chunk_rows):
            n = min(chunk_rows, self.R - a)
            chunk = torch.from_numpy(np.ascontiguousarray(rows[a:a + n])).to(self.device)
            self.kern.pack(chunk, self.board[a:a + n], flag)
        if int(flag.item()):
            raise ValueError(f"{path}: bytes other than 0/255 (use the single-GPU engine for those)")
        self.band = False
        self.halo_ok = False
        self.turn = 0

    # ------------------------------------------------------------ stepping
    def halo(self, k: int):
        """(top, bot): the k halo rows right above row 0 and right below row R-1 of buf[cur]."""
        st, km, R = self._store[self.cur], self.kmax, self.R
        return st[km - k:km], st[km + R:km + R + k]

    def _rows(self, row: int, rows: int) -> torch.Tensor:
        """Shard-local rows [row, row + rows) of buf[cur], ghost rows (row < 0 or >= R) included."""
        return self._store[self.cur][self.kmax + row:self.kmax + row + rows]

    def _exchange(self) -> None:
        """The library's halo plan (gol_halo_plan, the schedule libgolhip.so's engine runs) for
        this rank, kmax rows each way, in its issue order as torch.distributed P2P ops: a
        receiver's n-th receive from a peer meets that peer's n-th send to it (for two ranks one
        peer on both sides).  One rank: the plan's sends to itself, paired the same way (the
        torus wrap)."""
        plan = halo_plan(self.H, self.nranks, self.rank, self.kmax)
        if self.nranks == 1:
            sends = [self._rows(row, n).clone() for kind, _, row, n in plan if kind == "send"]
            recvs = [(row, n) for kind, _, row, n in plan if kind == "recv"]
            for (row, n), src in zip(recvs, sends):
                self._rows(row, n).copy_(src)
            return
        g = self.group
        stage = self.device.type == "cuda" and dist.get_backend(g) == "gloo"
        ops, land = [], []
        for kind, peer, row, n in plan:
            t = self._rows(row, n)
            if stage:
                # gloo has no device P2P: stage the halo rows through host memory (several ranks
                # sharing one GPU in tests; production runs RCCL inside libgolhip.so)
                buf = t.cpu() if kind == "send" else torch.empty(t.shape, dtype=t.dtype)
                if kind == "recv":
                    land.append((t, buf))
                t = buf
            elif kind == "recv" and not t.is_contiguous():
                buf = torch.empty_like(t)
                land.append((t, buf))
                t = buf
            ops.append(dist.P2POp(dist.isend if kind == "send" else dist.irecv, t, peer, g))
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        for dst, buf in land:
            dst.copy_(buf)

    def _launch(self, kind, top, bot, dst, row0, rows, k, slots):
        if rows <= 0:
            return
        hook = self.launch_hook
        if hook is not None:
            hook(kind, k, rows, True)
        step = self.kern.band_step if self.band else self.kern.bits_step
        step(top, self.board, bot, dst, row0, rows, k, slots)
        if hook is not None:
            hook(kind, k, rows, False)

    def step(self, turns: int, count: bool = False) -> None:
        """Advance exactly `turns` turns: per k-turn step the launches of the library's step plan
        (gol_step_plan: the edge rows, which read the halo, and the interior), then the next
        step's halo exchange (gol_halo_plan, kmax rows)."""
        if turns > 0 and self.use_band:
            self._convert(True)
        if turns > 0 and not self.halo_ok:
            self._exchange()
        while turns > 0:
            k = max(kk for kk in self.valid_k if kk <= min(self.kmax, turns))
            last = turns == k
            slots = self.slots if (count and last) else None
            if slots is not None:
                slots.zero_()
            dst = self.buf[1 - self.cur]
            top, bot = self.halo(k)
            for stream, _, row0, rows in step_plan(self.R, k, self.kmax):
                self._launch("edge" if stream == "edge" else "main", top, bot, dst, row0, rows, k, slots)
            self.cur = 1 - self.cur
            self._exchange()
            self.halo_ok = True
            self.turn += k
            turns -= k

    # ------------------------------------------------------------ queries
    def _allreduce(self, t: torch.Tensor) -> int:
        if self.nranks > 1:
            dist.all_reduce(t, group=self.group)
        return int(t.item()) & (2**64 - 1)

    def _slot_sum(self) -> torch.Tensor:
        return self.slots.view(GOL_COUNT_SLOTS, 8)[:, 0].sum().reshape(1)

    def alive_count(self) -> int:
        self.slots.zero_()
        self.kern.popcount(self.board, self.slots)
        return self._allreduce(self._slot_sum())

    def fused_count(self) -> int:
        """Alive count accumulated by the last launch of the last step(count=True)."""
        return self._allreduce(self._slot_sum())

    def hash(self) -> int:
        """Order-independent board hash (oracle_hash_words), summed over shards."""
        self.slots.zero_()
        self.kern.hash(self.standard(), self.y0, self.slots)
        return self._allreduce(self._slot_sum())

    def gather_bytes(self):
        """Whole board as (H, W) uint8 0/255 on rank 0 (None elsewhere).  Small boards only."""
        mine = self.kern.unpack(self.standard(), self.W)
        if self.nranks == 1:
            return mine.cpu()
        parts = [torch.empty((partition_rows(self.H, self.nranks, r)[1] - partition_rows(self.H, self.nranks, r)[0],
                              self.W), dtype=torch.uint8, device=mine.device) for r in range(self.nranks)]
        if self.rank == 0:
            parts[0].copy_(mine)
            for r in range(1, self.nranks):
                dist.recv(parts[r], r, group=self.group)
            return torch.cat([p.cpu() for p in parts])
        dist.send(mine, 0, group=self.group)
        return None


def _pgm_header(W: int, H: int) -> bytes:
    """gol/io.go:52-59: "P5\\n<W> <H>\\n255\\n"."""
    return b"P5\n%d %d\n255\n" % (W, H)


def stream_pgm(board: ShardedBoard, sink, chunk_rows: int = 4096) -> None:
    """Stream the board as the reference's P5 byte layout (gol/io.go:42-87) to `sink` on rank 0.

    Every rank unpacks its rows chunk by chunk on its GPU (bits -> 0/255 bytes) and sends them
    to rank 0 in row order; rank 0 copies each chunk to the host and calls sink(bytes).  No rank
    ever holds more than one chunk of bytes, so a 2^20 x 2^20 board (1 TiB of P5) streams with
    O(chunk) memory.  `sink` is only called on rank 0 (e.g. file.write or hashlib's update)."""
    W = board.W
    rows = board.standard()
    if board.rank == 0:
        sink(_pgm_header(W, board.H))
    for r in range(board.nranks):
        y0, y1 = partition_rows(board.H, board.nranks, r)
        for a in range(0, y1 - y0, chunk_rows):
            n = min(chunk_rows, y1 - y0 - a)
            if r == board.rank:
                part = board.kern.unpack(rows[a:a + n], W)
                if r != 0:
                    dist.send(part, 0, group=board.group)
                    continue
            elif board.rank == 0:
                part = torch.empty((n, W), dtype=torch.uint8, device=board.device)
                dist.recv(part, r, group=board.group)
            else:
                continue
            sink(part.cpu().numpy().tobytes())


def write_pgm(board: ShardedBoard, path: str, chunk_rows: int = 4096) -> None:
    """Write out/<W>x<H>x<Turns>.pgm-style P5 file from a sharded board (rank 0 writes)."""
    if board.rank == 0:
        with open(path, "wb") as f:
            stream_pgm(board, f.write, chunk_rows)
    else:
        stream_pgm(board, lambda b: None, chunk_rows)
