"""CPU oracle for the Game-of-Life hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this module, and only as the checker (or the timed CPU baseline).
The product (``golhip`` + ``libgolhip.so``) never imports it.

It wraps ``oracle/gol_oracle.c`` (built to ``oracle/liboracle.so``) and adds a
small numpy restatement plus the PGM codec of the reference:

* ``next_state_slab``   worker.go:15-70 (literal per-cell port, C)
* ``run``               broker.go:62-234 turn loop with the Threads slab split
* ``partition``         broker.go:135-139, 172-206
* ``alive_cells``       broker.go:47-58
* ``read_pgm``          gol/io.go:90-126 (strings.Fields parsing)
* ``pgm_bytes``         gol/io.go:42-87  ("P5\\n<W> <H>\\n255\\n" + H*W bytes)
* ``np_next_state``     numpy restatement of the same rule (cross-check)
* ``bits_run``          word-parallel restatement for long runs
* ``to_band`` / ``from_band``  the column-band bit layout (numpy restatement)

Pinned against the reference's own fixtures in ``tests/golden`` (copied from
/root/reference/check and /root/reference/images); see tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

i64 = ctypes.c_int64
u64 = ctypes.c_uint64
P = ctypes.c_void_p


def build() -> str:
    """Compile oracle/gol_oracle.c with gcc (make)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "gol_oracle.c")
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_count_neighbours.argtypes = [P, i64, i64, i64, i64, i64]
        L.oracle_count_neighbours.restype = ctypes.c_int
        L.oracle_next_state_slab.argtypes = [P, i64, i64, i64, i64, i64, P, i64]
        L.oracle_next_state_slab.restype = ctypes.c_int
        L.oracle_partition.argtypes = [i64, i64, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)]
        L.oracle_partition.restype = ctypes.c_int
        L.oracle_alive_cells.argtypes = [P, i64, i64, i64, P, i64]
        L.oracle_alive_cells.restype = i64
        L.oracle_run.argtypes = [P, i64, i64, i64, i64]
        L.oracle_run.restype = ctypes.c_int
        L.oracle_splitmix64.argtypes = [u64]
        L.oracle_splitmix64.restype = u64
        L.oracle_random_words.argtypes = [u64, i64, i64, i64, P]
        L.oracle_random_words.restype = None
        L.oracle_hash_words.argtypes = [P, i64, i64, i64]
        L.oracle_hash_words.restype = u64
        L.oracle_popcount_words.argtypes = [P, i64]
        L.oracle_popcount_words.restype = u64
        L.oracle_pack.argtypes = [P, i64, i64, i64, P]
        L.oracle_pack.restype = None
        L.oracle_unpack.argtypes = [P, i64, i64, P, i64]
        L.oracle_unpack.restype = None
        L.oracle_bits_run.argtypes = [P, i64, i64, i64, P]
        L.oracle_bits_run.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- literal port
def next_state_slab(world: np.ndarray, y0: int, y1: int) -> np.ndarray:
    """worker.go:15-42 calculateNextState(startY, endY, world) -> slab bytes."""
    world = np.ascontiguousarray(world, dtype=np.uint8)
    H, W = world.shape
    out = np.zeros((y1 - y0, W), dtype=np.uint8)
    rc = lib().oracle_next_state_slab(_ptr(world), H, W, W, y0, y1, _ptr(out), W)
    if rc != 0:
        raise ValueError("bad slab bounds")
    return out


def run(world: np.ndarray, turns: int, threads: int = 1) -> np.ndarray:
    """broker.go:62-234 Operations.Run: `turns` turns with `threads` slabs per turn."""
    w = np.array(world, dtype=np.uint8, order="C", copy=True)
    H, W = w.shape
    rc = lib().oracle_run(_ptr(w), H, W, turns, threads)
    if rc != 0:
        raise ValueError("oracle_run failed")
    return w


def partition(H: int, threads: int, i: int) -> tuple[int, int]:
    """broker.go:135-139 / 172-206 row split -> (StartY, EndY)."""
    a, b = i64(), i64()
    if lib().oracle_partition(H, threads, i, ctypes.byref(a), ctypes.byref(b)) != 0:
        raise ValueError("bad partition arguments")
    return a.value, b.value


def alive_cells(world: np.ndarray) -> list[tuple[int, int]]:
    """broker.go:47-58 calculateAliveCells -> [(X, Y)] row-major, bytes != 0."""
    world = np.ascontiguousarray(world, dtype=np.uint8)
    H, W = world.shape
    n = int(np.count_nonzero(world))
    xy = np.zeros(2 * max(n, 1), dtype=np.int64)
    got = lib().oracle_alive_cells(_ptr(world), H, W, W, _ptr(xy), n)
    assert got == n
    return [(int(xy[2 * i]), int(xy[2 * i + 1])) for i in range(n)]


def flipped_cells(prev: np.ndarray, cur: np.ndarray) -> list[tuple[int, int]]:
    """CellFlipped events of one turn (gol/event.go:50-60: one event per cell whose state
    changed between CompletedTurns-1 and CompletedTurns), row-major [(X, Y)] like
    calculateAliveCells (broker.go:47-58); alive = byte != 0."""
    ys, xs = np.nonzero((np.asarray(prev) != 0) != (np.asarray(cur) != 0))
    return list(zip(xs.tolist(), ys.tolist()))


# ---------------------------------------------------------------- numpy restatement
def np_next_state(world: np.ndarray) -> np.ndarray:
    """Same rule as worker.go:15-70, vectorised: count of ==255 neighbours on
    the torus; ==0 with 3 -> 255; ==255 with 2 or 3 -> 255; everything else 0."""
    alive = (world == 255).astype(np.uint8)
    n = np.zeros(world.shape, dtype=np.uint8)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy or dx:
                n += np.roll(np.roll(alive, dy, axis=0), dx, axis=1)
    out = np.zeros_like(world)
    out[(world == 0) & (n == 3)] = 255
    out[(world == 255) & ((n == 2) | (n == 3))] = 255
    return out


# ---------------------------------------------------------------- bit-packed restatement
def random_words(seed: int, y0: int, rows: int, Ww: int) -> np.ndarray:
    out = np.zeros((rows, Ww), dtype=np.uint64)
    lib().oracle_random_words(seed, y0, rows, Ww, _ptr(out))
    return out


def hash_words(words: np.ndarray, y0: int = 0) -> int:
    words = np.ascontiguousarray(words, dtype=np.uint64)
    rows, Ww = words.shape
    return int(lib().oracle_hash_words(_ptr(words), y0, rows, Ww))


def popcount_words(words: np.ndarray) -> int:
    words = np.ascontiguousarray(words, dtype=np.uint64)
    return int(lib().oracle_popcount_words(_ptr(words), words.size))


def pack(board: np.ndarray) -> np.ndarray:
    board = np.ascontiguousarray(board, dtype=np.uint8)
    H, W = board.shape
    assert W % 64 == 0
    out = np.zeros((H, W // 64), dtype=np.uint64)
    lib().oracle_pack(_ptr(board), H, W, W, _ptr(out))
    return out


def unpack(words: np.ndarray) -> np.ndarray:
    words = np.ascontiguousarray(words, dtype=np.uint64)
    H, Ww = words.shape
    out = np.zeros((H, Ww * 64), dtype=np.uint8)
    lib().oracle_unpack(_ptr(words), H, Ww * 64, _ptr(out), Ww * 64)
    return out


def bits_run(words: np.ndarray, turns: int, with_counts: bool = False):
    w = np.array(words, dtype=np.uint64, order="C", copy=True)
    H, Ww = w.shape
    counts = np.zeros(max(turns, 1), dtype=np.int64)
    rc = lib().oracle_bits_run(_ptr(w), H, Ww, turns, _ptr(counts) if with_counts else None)
    if rc != 0:
        raise ValueError("oracle_bits_run failed")
    return (w, counts[:turns]) if with_counts else w


# ------------------------------------------ the same restatement, multi-threaded and in place
# (oracle/gol_oracle_mt.c -> liboracle_mt.so): the count series of full-size boards
# (tools/pin_counts_oracle.py), cross-checked against bits_run in tests/test_oracle.py.
_MT_PATH = os.path.join(_HERE, "liboracle_mt.so")
_mt = None


def mt_lib():
    global _mt
    if _mt is None:
        src = os.path.join(_HERE, "gol_oracle_mt.c")
        if not os.path.exists(_MT_PATH) or os.path.getmtime(_MT_PATH) < os.path.getmtime(src):
            build()
        L = ctypes.CDLL(_MT_PATH)
        L.oracle_mt_bits_run.argtypes = [P, i64, i64, i64, i64, P, ctypes.c_int]
        L.oracle_mt_bits_run.restype = ctypes.c_int
        L.oracle_mt_random_words.argtypes = [u64, i64, i64, P, ctypes.c_int]
        L.oracle_mt_random_words.restype = None
        L.oracle_mt_hash_words.argtypes = [P, i64, i64, ctypes.c_int]
        L.oracle_mt_hash_words.restype = u64
        _mt = L
    return _mt


def mt_random_words(seed: int, H: int, Ww: int, threads: int = 8) -> np.ndarray:
    """random_words(seed, 0, H, Ww), filled by `threads` threads."""
    out = np.empty((H, Ww), dtype=np.uint64)
    mt_lib().oracle_mt_random_words(seed, H, Ww, _ptr(out), threads)
    return out


def mt_hash_words(words: np.ndarray, threads: int = 8) -> int:
    assert words.dtype == np.uint64 and words.flags.c_contiguous
    H, Ww = words.shape
    return int(mt_lib().oracle_mt_hash_words(_ptr(words), H, Ww, threads))


def mt_bits_run(words: np.ndarray, turns: int, every: int = 1, threads: int = 8) -> np.ndarray:
    """`turns` generations IN PLACE on `words` (C-contiguous uint64 rows); returns the alive
    counts after turns every, 2*every, ... (turns // every of them)."""
    assert words.dtype == np.uint64 and words.flags.c_contiguous and words.ndim == 2
    H, Ww = words.shape
    counts = np.zeros(max(turns // every, 1), dtype=np.int64)
    rc = mt_lib().oracle_mt_bits_run(_ptr(words), H, Ww, turns, every, _ptr(counts), threads)
    if rc != 0:
        raise ValueError("oracle_mt_bits_run failed")
    return counts[: turns // every]


def to_band(words: np.ndarray) -> np.ndarray:
    """Standard bit rows (uint64, 64 cells per word) -> band rows as uint32 words:
    band word w of a row holds at bit b the cell x = b*Wd + w (Wd = W/32).  This is
    the layout definition of gol_dev_band_convert, restated."""
    cells = unpack(words) != 0                      # (H, W) bool, x = column
    H, W = cells.shape
    Wd = W // 32
    bands = cells.reshape(H, 32, Wd).astype(np.uint64)  # [y, b, w]
    shifts = np.arange(32, dtype=np.uint64)[None, :, None]
    return (bands << shifts).sum(axis=1).astype(np.uint32)


def from_band(band: np.ndarray) -> np.ndarray:
    """Inverse of to_band: band uint32 rows -> standard uint64 rows."""
    band = np.ascontiguousarray(band, dtype=np.uint32)
    H, Wd = band.shape
    bits = (band[:, None, :] >> np.arange(32, dtype=np.uint32)[None, :, None]) & 1  # [y, b, w]
    cells = bits.reshape(H, 32 * Wd).astype(np.uint8) * 255
    return pack(cells)


# ---------------------------------------------------------------- PGM codec (gol/io.go)
_GO_SPACE = b" \t\n\v\f\r"


def read_pgm(path: str, width: int | None = None, height: int | None = None):
    """gol/io.go:90-126 readPgmImage: strings.Fields(data); fields[0] == "P5",
    fields[1] == width, fields[2] == height, fields[3] == 255, pixels = fields[4].
    Returns (W, H, board[H, W])."""
    with open(path, "rb") as f:
        data = f.read()
    # strings.Fields splits on unicode.IsSpace; for the bytes that can occur in
    # these files (0, 255 and ASCII header text) that is the ASCII set above
    # plus U+0085/U+00A0, which cannot appear as single invalid-UTF-8 bytes.
    fields = []
    i, n = 0, len(data)
    while i < n and len(fields) < 5:
        while i < n and data[i] in _GO_SPACE:
            i += 1
        j = i
        while j < n and data[j] not in _GO_SPACE:
            j += 1
        if j > i:
            fields.append(data[i:j])
        i = j
    if not fields or fields[0] != b"P5":
        raise ValueError("Not a pgm file")
    W, H, maxval = int(fields[1]), int(fields[2]), int(fields[3])
    if width is not None and W != width:
        raise ValueError("Incorrect width")
    if height is not None and H != height:
        raise ValueError("Incorrect height")
    if maxval != 255:
        raise ValueError("Incorrect maxval/bit depth")
    pix = np.frombuffer(fields[4], dtype=np.uint8)
    if pix.size != W * H:
        raise ValueError("pixel data is not W*H bytes")
    return W, H, pix.reshape(H, W).copy()


def pgm_bytes(board: np.ndarray) -> bytes:
    """gol/io.go:52-81 writePgmImage byte stream."""
    H, W = board.shape
    return b"P5\n" + str(W).encode() + b" " + str(H).encode() + b"\n" + b"255\n" + \
        np.ascontiguousarray(board, dtype=np.uint8).tobytes()


def read_alive_csv(path: str) -> dict[int, int]:
    """count_test.go:71-89 readAliveCounts -> {completed_turns: alive}."""
    out = {}
    with open(path) as f:
        for i, line in enumerate(f):
            if i == 0 or not line.strip():
                continue
            t, c = line.strip().split(",")
            out[int(t)] = int(c)
    return out
