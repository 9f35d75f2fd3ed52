"""Row-sharded board over several ranks with the gloo backend on CPU.

Checks the host logic of golhip.sharded.ShardedBoard -- the broker.go:172-206
partition applied to ranks, ghost-row layout, the halo exchange order (including
N=2, where both neighbours are the same peer), uneven shards and k-turn chunks --
against the oracle on the whole torus.  The GPU kernels are replaced here by a
CPU stand-in built on the oracle (test-only; the product has no CPU path).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O


class OracleKernels:
    """CPU stand-in for golhip.sharded.HipKernels with the same tensor interface."""

    @staticmethod
    def _words(t):
        a = t.numpy().view(np.uint32)
        return a

    def bits_step(self, top, mid, bot, dst, row0, rows, k, slots=None):
        R = mid.shape[0]
        Wd = self.Wd
        rows_in = []
        for y in range(row0 - k, row0 + rows + k):
            if y < 0:
                src = top[y + k]
            elif y >= R:
                src = bot[y - R]
            else:
                src = mid[y]
            rows_in.append(src.numpy().view(np.uint32)[:Wd])
        stack = np.ascontiguousarray(np.stack(rows_in)).view(np.uint64)
        out = O.bits_run(stack, k)[k:k + rows]
        dst.numpy().view(np.uint32)[row0:row0 + rows, :Wd] = np.ascontiguousarray(out).view(np.uint32)
        if slots is not None:
            slots[0] += O.popcount_words(out)

    def band_step(self, top, mid, bot, dst, row0, rows, k, slots=None):
        # same as bits_step on the band layout: restate through the standard layout
        R = mid.shape[0]
        Wd = self.Wd
        rows_in = []
        for y in range(row0 - k, row0 + rows + k):
            src = top[y + k] if y < 0 else (bot[y - R] if y >= R else mid[y])
            rows_in.append(src.numpy().view(np.uint32)[:Wd])
        std = O.from_band(np.stack(rows_in))
        out = O.bits_run(std, k)[k:k + rows]
        dst.numpy().view(np.uint32)[row0:row0 + rows, :Wd] = O.to_band(out)
        if slots is not None:
            slots[0] += O.popcount_words(out)

    def band_convert(self, to_band, src, dst):
        a = np.ascontiguousarray(src.numpy().view(np.uint32)[:, :self.Wd])
        if to_band:
            dst.numpy().view(np.uint32)[:, :self.Wd] = O.to_band(a.view(np.uint64))
        else:
            dst.numpy().view(np.uint32)[:, :self.Wd] = O.from_band(a).view(np.uint32)

    def random_fill(self, dst, grow0, W, seed):
        rows = dst.shape[0]
        words = O.random_words(seed, grow0, rows, W // 64)
        dst.numpy().view(np.uint32)[:, :W // 32] = words.view(np.uint32)

    def popcount(self, src, slots):
        slots[0] += O.popcount_words(np.ascontiguousarray(src.numpy().view(np.uint32)[:, :self.Wd]).view(np.uint64))

    def hash(self, src, grow0, slots):
        w = np.ascontiguousarray(src.numpy().view(np.uint32)[:, :self.Wd]).view(np.uint64)
        h = O.hash_words(w, grow0)
        slots[0] += int(np.array(h, dtype=np.uint64).view(np.int64))

    def unpack(self, src, W):
        w = np.ascontiguousarray(src.numpy().view(np.uint32)[:, :self.Wd]).view(np.uint64)
        return torch.from_numpy(O.unpack(w))

    def pack(self, board, dst, nonbinary=None):
        b = board.numpy()
        dst.numpy().view(np.uint32)[:, :self.Wd] = O.pack(b).view(np.uint32)
        if nonbinary is not None and ((b != 0) & (b != 255)).any():
            nonbinary[0] = 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, H, W, k, turns, seed, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golhip.sharded import ShardedBoard
        b = ShardedBoard(H, W, turns_per_launch=k, kernels=OracleKernels(), device="cpu")
        assert b.use_band == (W % 1024 == 0)
        b.load_random(seed)
        h0 = b.hash()
        b.step(turns, count=True)
        fused = b.fused_count()
        out = (rank, b.y0, b.y1, b.kmax, h0, b.hash(), b.alive_count(), fused)
        full = b.gather_bytes()
        import hashlib
        from golhip.sharded import stream_pgm
        h = hashlib.sha256()
        stream_pgm(b, h.update, chunk_rows=3)
        q.put(out + ((full.numpy() if full is not None else None), h.hexdigest() if rank == 0 else None))
    finally:
        dist.destroy_process_group()


def _run(world, H, W, k, turns, seed=5):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, k, turns, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


@pytest.mark.parametrize("world,H,W,k,turns", [(2, 64, 128, 8, 21), (3, 50, 128, 4, 13), (4, 67, 128, 2, 9),
                                                (2, 9, 128, 4, 6),
                                                # W % 1024 == 0: stepped in the band layout
                                                (2, 40, 1024, 8, 19), (3, 31, 2048, 4, 11)])
def test_sharded_matches_oracle(world, H, W, k, turns):
    words = O.random_words(5, 0, H, W // 64)
    ref = O.bits_run(words, turns)
    res = _run(world, H, W, k, turns)
    for r, (rank, y0, y1, kmax, h0, h1, count, fused, full, digest) in enumerate(res):
        assert (y0, y1) == O.partition(H, world, rank)       # broker.go:172-206 split
        assert kmax <= H // world
        assert h0 == O.hash_words(words)                     # same global board for any N
        assert h1 == O.hash_words(ref)
        assert count == fused == O.popcount_words(ref)
    assert np.array_equal(res[0][-2], O.unpack(ref))
    import hashlib
    assert res[0][-1] == hashlib.sha256(O.pgm_bytes(O.unpack(ref))).hexdigest()  # gol/io.go P5 bytes


def _pgm_worker(rank, world, port, path, W, H, turns, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golhip.sharded import ShardedBoard
        b = ShardedBoard(H, W, turns_per_launch=8, kernels=OracleKernels(), device="cpu")
        b.load_pgm(path, chunk_rows=7)  # odd chunks: several per shard
        b.step(turns)
        full = b.gather_bytes()
        q.put((rank, full.numpy() if full is not None else None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_load_pgm_golden(world, golden_dir):
    """Each rank streams only its rows of images/512x512.pgm (memory-mapped, gol/io.go header
    rules); 100 turns on the sharded board reproduce check/images/512x512x100.pgm."""
    path = os.path.join(golden_dir, "images", "512x512.pgm")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pgm_worker, args=(r, world, port, path, 512, 512, 100, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    _, _, want = O.read_pgm(os.path.join(golden_dir, "check", "images", "512x512x100.pgm"))
    assert np.array_equal(res[0], want)


def test_pgm_rows_header_rules(tmp_path):
    """golhip.pgm.pgm_rows: header rules of gol/io.go:98-119 and row windows of the raster."""
    from golhip._lib import GolError
    from golhip.pgm import pgm_rows
    board = (np.arange(6 * 8).reshape(6, 8) % 2 * 255).astype(np.uint8)
    p = tmp_path / "b.pgm"
    p.write_bytes(O.pgm_bytes(board))
    assert np.array_equal(np.asarray(pgm_rows(str(p), 2, 5)), board[2:5])
    assert np.array_equal(np.asarray(pgm_rows(str(p), 0, 6, 8, 6)), board)
    with pytest.raises(GolError):
        pgm_rows(str(p), 0, 1, width=9)
    bad = tmp_path / "bad.pgm"
    bad.write_bytes(b"P6\n8 6\n255\n" + board.tobytes())
    with pytest.raises(GolError):
        pgm_rows(str(bad), 0, 1)
    short = tmp_path / "short.pgm"
    short.write_bytes(O.pgm_bytes(board)[:-3])
    with pytest.raises(GolError):
        pgm_rows(str(short), 0, 1)
